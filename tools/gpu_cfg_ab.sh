# Configs 3 and 5 (tools/bench_configs.py, 10 passes) with an older build
# (GPURAFT_LIB) beside the current one on the same box, then the config kernel
# trace and config-5 counters of the current build (tools/profile_configs.sh).
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for lib in libgpuraft_r03.so libgpuraft.so; do
  GPURAFT_LIB=$PWD/dragonboat_amd/_build/$lib timeout -k 10 300 python -u tools/bench_configs.py --passes 10 --only 3,5 > gpurun_out/cfg_$lib.json 2> gpurun_out/cfg_$lib.err || { tail -5 gpurun_out/cfg_$lib.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/cfg_$lib.json'):
    d=json.loads(l); print('$lib', d['config'][:12], '%.1f us' % (d['device_ms_per_pass']*1e3), 'fast %.1f gen %.1f' % (d['fast_ms']*1e3, d['general_ms']*1e3), 'bailed', d['bailed_lanes_per_pass'], 'esc/pass', d['escalations_per_pass'])
"
done
TAG=r04_a ONLY=2,3,5 PMC_ONLY=3,5 bash tools/profile_configs.sh > gpurun_out/profcfg.log 2>&1 || { tail -20 gpurun_out/profcfg.log; exit 1; }
python -c "
import json
d=json.load(open('gpurun_out/cfgprof_r04_a/summary.json'))
for k,v in d['trace'].items(): print(k, round(v['avg_us'],1), round(v['min_us'],1), v['launches'])
"
