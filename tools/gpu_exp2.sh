# After the H_MP fix: headline bench first, then device-schedule parity, then
# config experiments (config 2 padded layout, config 5 general binning).
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/exp_bench.json 2> gpurun_out/exp_bench.err || { tail -5 gpurun_out/exp_bench.err; exit 1; }
python -c "
import json
d=json.loads(open('gpurun_out/exp_bench.json').read().strip().splitlines()[-1])
r=d['roofline']; print('bench', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('general_kernel_ms'), d['host_path']['ms_per_pass'])
"
timeout -k 10 600 python -u -m pytest tests/test_device_schedule.py tests/test_gpu.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/exp_tests.log 2>&1 || { tail -30 gpurun_out/exp_tests.log; exit 1; }
tail -2 gpurun_out/exp_tests.log
for g in 10000 10048; do
  timeout -k 10 200 python -u tools/bench_configs.py --passes 20 --only 2 --groups2 $g > gpurun_out/exp_c2_$g.json 2> gpurun_out/exp_c2_$g.err || { tail -5 gpurun_out/exp_c2_$g.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/exp_c2_$g.json').read().strip().splitlines()[-1])
print('$g', '%.1f us events' % (d['device_ms_per_pass']*1e3), 'graph %.1f us' % (d['graph']['ms_per_pass']*1e3))
"
done
for b in 0 1; do
  GR_BIN_GENERAL=$b GR_WAVE_CLOCK=gpurun_out/wc5_$b.bin timeout -k 10 300 python -u tools/bench_configs.py --passes 10 --only 3,5 > gpurun_out/exp_c35_$b.json 2> gpurun_out/exp_c35_$b.err || { tail -5 gpurun_out/exp_c35_$b.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/exp_c35_$b.json'):
    d=json.loads(l); print('bin $b', d['config'][:12], '%.1f us' % (d['device_ms_per_pass']*1e3), 'fast %.1f gen %.1f bailed %d' % (d['fast_ms']*1e3, d['general_ms']*1e3, d['bailed_lanes_per_pass']))
"
  python tools/wave_clock.py gpurun_out/wc5_$b.bin | head -4
done
