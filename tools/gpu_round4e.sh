# Parity of the device schedule (class appends in one atomic round), config
# evidence (tools/profile_configs.sh: trace of configs 2, 3, 5, PMC of 3 and 5),
# then the launch-mode A/B of the headline.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_device_schedule.py tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/e_tests.log 2>&1 || { tail -30 gpurun_out/e_tests.log; exit 1; }
tail -1 gpurun_out/e_tests.log
TAG=r04_b bash tools/profile_configs.sh > gpurun_out/profcfg.log 2>&1 || { tail -20 gpurun_out/profcfg.log; exit 1; }
python -c "
import json
for l in open('gpurun_out/cfgprof_r04_b/configs.json'):
    d=json.loads(l); print(d['config'][:12], '%.1f us' % (d['device_ms_per_pass']*1e3), 'fast %.1f gen %.1f bailed %d' % (d['fast_ms']*1e3, d['general_ms']*1e3, d['bailed_lanes_per_pass']), d.get('graph', {}).get('ms_per_pass'))
"
bash tools/gpu_launch_ab.sh
