# Final evidence for the final build: -m gpu suite + smoke, bench line,
# tools/profile.sh (TAG r04_i: PMC for this digest), config 5 A/B against the
# previous build (lazy remote rows for non-leader general lanes), configs at 10 passes.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
TAG=r04_i bash tools/gpu_round.sh || exit $?
for i in 1 2; do
  for v in prev new; do
    if [ $v = prev ]; then export GPURAFT_LIB=$GRAFT_REPO_ROOT/dragonboat_amd/_build/ab/libgpuraft_prev.so; else unset GPURAFT_LIB; fi
    timeout -k 10 300 python -u tools/bench_configs.py --passes 10 --only 5 > gpurun_out/ab/r_$v$i.json 2> gpurun_out/ab/r_$v$i.err || { tail -5 gpurun_out/ab/r_$v$i.err; exit 1; }
    python -c "
import json
d=json.loads(open('gpurun_out/ab/r_$v$i.json').read().strip().splitlines()[-1]); print('$v$i', '%.1f us' % (d['device_ms_per_pass']*1e3), 'fast %.1f gen %.1f' % (d['fast_ms']*1e3, d['general_ms']*1e3))
"
  done
done
unset GPURAFT_LIB
timeout -k 10 400 python -u tools/bench_configs.py --passes 10 > gpurun_out/final_configs10.json 2> gpurun_out/final_configs10.err || { tail -5 gpurun_out/final_configs10.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/final_configs10.json'):
    d=json.loads(l); print(d['config'][:12], '%.1f us' % (d['device_ms_per_pass']*1e3), 'fast %.1f gen %.1f bailed %d' % (d['fast_ms']*1e3, d['general_ms']*1e3, d['bailed_lanes_per_pass']), d.get('graph', {}).get('ms_per_pass'))
"
