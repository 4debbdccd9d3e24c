# Parity of the device schedule first, then experiments: config 2 at 10,000 vs
# 10,048 groups (mixed leader/follower waves at the replica-block boundaries),
# configs 3/5, and the headline bench line.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_device_schedule.py tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/exp_tests.log 2>&1 || { tail -30 gpurun_out/exp_tests.log; exit 1; }
tail -2 gpurun_out/exp_tests.log
for g in 10000 10048; do
  timeout -k 10 200 python -u tools/bench_configs.py --passes 20 --only 2 --groups2 $g > gpurun_out/exp_c2_$g.json 2> gpurun_out/exp_c2_$g.err || { tail -5 gpurun_out/exp_c2_$g.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/exp_c2_$g.json').read().strip().splitlines()[-1])
print('$g', '%.1f us events' % (d['device_ms_per_pass']*1e3), 'graph %.1f us' % (d['graph']['ms_per_pass']*1e3))
"
done
timeout -k 10 300 python -u tools/bench_configs.py --passes 10 --only 3,5 > gpurun_out/exp_c35.json 2> gpurun_out/exp_c35.err || { tail -5 gpurun_out/exp_c35.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/exp_c35.json'):
    d=json.loads(l); print(d['config'][:12], '%.1f us' % (d['device_ms_per_pass']*1e3), 'fast %.1f gen %.1f' % (d['fast_ms']*1e3, d['general_ms']*1e3))
"
timeout -k 10 300 python -u bench.py > gpurun_out/exp_bench.json 2> gpurun_out/exp_bench.err || { tail -5 gpurun_out/exp_bench.err; exit 1; }
python -c "
import json
d=json.loads(open('gpurun_out/exp_bench.json').read().strip().splitlines()[-1])
print('bench', d['value'], d['ms_per_step'], d['roofline'])
"
GR_WAVE_CLOCK=gpurun_out/wc5.bin timeout -k 10 200 python -u tools/bench_configs.py --passes 6 --only 5 > gpurun_out/exp_wc5.json 2> gpurun_out/exp_wc5.err || { tail -5 gpurun_out/exp_wc5.err; exit 1; }
python tools/wave_clock.py gpurun_out/wc5.bin
GR_BIN_GENERAL=1 GR_WAVE_CLOCK=gpurun_out/wc5b.bin timeout -k 10 200 python -u tools/bench_configs.py --passes 6 --only 5 > gpurun_out/exp_wc5b.json 2> gpurun_out/exp_wc5b.err || { tail -5 gpurun_out/exp_wc5b.err; exit 1; }
python tools/wave_clock.py gpurun_out/wc5b.bin
python -c "
import json
for f in ('exp_wc5', 'exp_wc5b'):
    d=json.loads(open('gpurun_out/%s.json' % f).read().strip().splitlines()[-1]); print(f, '%.1f us' % (d['device_ms_per_pass']*1e3), 'fast %.1f gen %.1f bailed %d' % (d['fast_ms']*1e3, d['general_ms']*1e3, d['bailed_lanes_per_pass']))
"
