# Dynamic general-kernel chunks: parity (device schedule + GPU suite subset),
# config 5 at 10 and 20 passes with the per-class wave clock, then the lean-kernel
# PMC for this source digest (tools/profile.sh r04_h).
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_device_schedule.py tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/i_tests.log 2>&1 || { tail -30 gpurun_out/i_tests.log; exit 1; }
tail -1 gpurun_out/i_tests.log
for P in 10 20; do
  GR_WAVE_CLOCK=gpurun_out/wc5_dyn$P.bin timeout -k 10 300 python -u tools/bench_configs.py --passes $P --only 5 > gpurun_out/c5_dyn$P.json 2> gpurun_out/c5_dyn$P.err || { tail -5 gpurun_out/c5_dyn$P.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/c5_dyn$P.json').read().strip().splitlines()[-1]); print('passes $P', '%.1f us' % (d['device_ms_per_pass']*1e3), 'fast %.1f gen %.1f bailed %d' % (d['fast_ms']*1e3, d['general_ms']*1e3, d['bailed_lanes_per_pass']))
"
  python tools/wave_clock.py gpurun_out/wc5_dyn$P.bin > gpurun_out/wc5_dyn$P.txt; sed -n 2,4p gpurun_out/wc5_dyn$P.txt
done
TAG=r04_h bash tools/profile.sh > gpurun_out/profile_h4.log 2>&1 || { tail -10 gpurun_out/profile_h4.log; exit 1; }
grep -A3 '"lean_kernel_bytes_per_pass"' gpurun_out/prof_r04_h/summary.json
