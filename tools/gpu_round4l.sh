# Final build (r04_h digest): -m gpu suite + smoke, the bench line, configs at 10 passes.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PROFILE=0 bash tools/gpu_round.sh || exit $?
timeout -k 10 400 python -u tools/bench_configs.py --passes 10 > gpurun_out/final_configs10.json 2> gpurun_out/final_configs10.err || { tail -5 gpurun_out/final_configs10.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/final_configs10.json'):
    d=json.loads(l); print(d['config'][:12], '%.1f us' % (d['device_ms_per_pass']*1e3), 'fast %.1f gen %.1f bailed %d' % (d['fast_ms']*1e3, d['general_ms']*1e3, d['bailed_lanes_per_pass']), d.get('graph', {}).get('ms_per_pass'))
"
