# Final-build config passes at r03's protocol (10 timed passes) and the spread
# placement at N = 1 beside local.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/bench_configs.py --passes 10 > gpurun_out/final_configs10.json 2> gpurun_out/final_configs10.err || { tail -5 gpurun_out/final_configs10.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/final_configs10.json'):
    d=json.loads(l); print(d['config'][:12], '%.1f us' % (d['device_ms_per_pass']*1e3), 'fast %.1f gen %.1f bailed %d' % (d['fast_ms']*1e3, d['general_ms']*1e3, d['bailed_lanes_per_pass']), d.get('graph', {}).get('ms_per_pass'))
"
for pl in local spread; do
  timeout -k 10 200 python -u bench.py --placement $pl --steps 40 --cpu-baseline off --host-path off > gpurun_out/final_$pl.json 2> gpurun_out/final_$pl.err || { tail -5 gpurun_out/final_$pl.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/final_$pl.json').read().strip().splitlines()[-1]); print('$pl', round(d['ms_per_step'],5), round(d['value']/1e9,3))"
done
