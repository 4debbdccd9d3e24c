# Compact pairs + 24-B results, class-keyed general lists: parity first
# (compact, wire path, device schedule, GPU suite), then config 5 A/B with wave
# clocks, config 2 aligned, the headline bench with the host path.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_compact.py tests/test_wire_path.py tests/test_device_schedule.py tests/test_gpu.py tests/test_coverage.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/exp_tests.log 2>&1 || { tail -40 gpurun_out/exp_tests.log; exit 1; }
tail -2 gpurun_out/exp_tests.log
for b in 0 1; do
  GR_BIN_GENERAL=$b GR_WAVE_CLOCK=gpurun_out/wc5_$b.bin timeout -k 10 300 python -u tools/bench_configs.py --passes 10 --only 5 > gpurun_out/exp_c5_$b.json 2> gpurun_out/exp_c5_$b.err || { tail -5 gpurun_out/exp_c5_$b.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/exp_c5_$b.json'):
    d=json.loads(l); print('bin $b', d['config'][:12], '%.1f us' % (d['device_ms_per_pass']*1e3), 'fast %.1f gen %.1f bailed %d' % (d['fast_ms']*1e3, d['general_ms']*1e3, d['bailed_lanes_per_pass']))
"
  python tools/wave_clock.py gpurun_out/wc5_$b.bin > gpurun_out/wc5_$b.txt; head -4 gpurun_out/wc5_$b.txt; grep phase gpurun_out/wc5_$b.txt || true
done
timeout -k 10 200 python -u tools/bench_configs.py --passes 20 --only 2 > gpurun_out/exp_c2.json 2> gpurun_out/exp_c2.err || { tail -5 gpurun_out/exp_c2.err; exit 1; }
python -c "
import json
d=json.loads(open('gpurun_out/exp_c2.json').read().strip().splitlines()[-1])
print('c2 aligned', d['lane_groups'], '%.1f us events' % (d['device_ms_per_pass']*1e3), 'graph %.1f us' % (d['graph']['ms_per_pass']*1e3))
"
timeout -k 10 300 python -u bench.py > gpurun_out/exp_bench.json 2> gpurun_out/exp_bench.err || { tail -5 gpurun_out/exp_bench.err; exit 1; }
python -c "
import json
d=json.loads(open('gpurun_out/exp_bench.json').read().strip().splitlines()[-1])
r=d['roofline']; h=d['host_path']; print('bench', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('general_kernel_ms'), 'host', h['ms_per_pass'], h['record_bytes_per_pass'])
"
