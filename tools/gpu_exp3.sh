# Class-keyed general lists + phase marks: parity (device schedule, GPU suite
# subset), then config 5 A/B (GR_BIN_GENERAL=0 vs the default) with wave clocks,
# then the headline bench.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_device_schedule.py tests/test_gpu.py tests/test_coverage.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/exp_tests.log 2>&1 || { tail -30 gpurun_out/exp_tests.log; exit 1; }
tail -2 gpurun_out/exp_tests.log
for b in 0 1; do
  GR_BIN_GENERAL=$b GR_WAVE_CLOCK=gpurun_out/wc5_$b.bin timeout -k 10 300 python -u tools/bench_configs.py --passes 10 --only 5 > gpurun_out/exp_c5_$b.json 2> gpurun_out/exp_c5_$b.err || { tail -5 gpurun_out/exp_c5_$b.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/exp_c5_$b.json'):
    d=json.loads(l); print('bin $b', d['config'][:12], '%.1f us' % (d['device_ms_per_pass']*1e3), 'fast %.1f gen %.1f bailed %d' % (d['fast_ms']*1e3, d['general_ms']*1e3, d['bailed_lanes_per_pass']))
"
  python tools/wave_clock.py gpurun_out/wc5_$b.bin > gpurun_out/wc5_$b.txt; head -4 gpurun_out/wc5_$b.txt; grep phase gpurun_out/wc5_$b.txt
done
timeout -k 10 300 python -u bench.py > gpurun_out/exp_bench.json 2> gpurun_out/exp_bench.err || { tail -5 gpurun_out/exp_bench.err; exit 1; }
python -c "
import json
d=json.loads(open('gpurun_out/exp_bench.json').read().strip().splitlines()[-1])
r=d['roofline']; print('bench', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('general_kernel_ms'), d['host_path']['ms_per_pass'])
"
