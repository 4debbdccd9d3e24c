# Round-4 final evidence: pytest -m gpu + smoke, the bench line, tools/profile.sh
# (TAG r04_d: trace + calibrated PMC, pmc_latest.json for this source digest), then
# the per-config device passes (tools/bench_configs.py defaults, untraced).
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=r04_d bash tools/gpu_round.sh || exit $?
timeout -k 10 400 python -u tools/bench_configs.py > gpurun_out/final_configs.json 2> gpurun_out/final_configs.err || { tail -5 gpurun_out/final_configs.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/final_configs.json'):
    d=json.loads(l); print(d['config'][:12], '%.1f us' % (d['device_ms_per_pass']*1e3), 'fast %.1f gen %.1f bailed %d' % (d['fast_ms']*1e3, d['general_ms']*1e3, d['bailed_lanes_per_pass']), d.get('graph', {}).get('ms_per_pass'))
"
