# The -m gpu suite + smoke, configs 2/3/5 (tools/bench_configs.py, 10 passes),
# the headline bench line.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit $?
timeout -k 10 300 python -u tools/bench_configs.py --passes 10 > gpurun_out/configs.json 2> gpurun_out/configs.err || { tail -5 gpurun_out/configs.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/configs.json'):
    d=json.loads(l); print(d['config'][:12], '%.1f us' % (d['device_ms_per_pass']*1e3), 'fast %.1f gen %.1f' % (d['fast_ms']*1e3, d['general_ms']*1e3), 'bailed', d['bailed_lanes_per_pass'], 'esc/pass', d['escalations_per_pass'], d.get('graph', {}).get('ms_per_pass'))
"
bash tools/ab_env.sh "A=local" > gpurun_out/ab_local.log 2>&1 || { cat gpurun_out/ab_local.log; exit 1; }
cat gpurun_out/ab_local.log
