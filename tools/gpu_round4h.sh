# Per-class wave clock of config 5's general kernel, parity of the device
# schedule, and the lean-kernel PMC for this source digest (tools/profile.sh r04_g).
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
GR_WAVE_CLOCK=gpurun_out/wc5_cls.bin timeout -k 10 300 python -u tools/bench_configs.py --passes 10 --only 5 > gpurun_out/c5_cls.json 2> gpurun_out/c5_cls.err || { tail -5 gpurun_out/c5_cls.err; exit 1; }
python tools/wave_clock.py gpurun_out/wc5_cls.bin > gpurun_out/wc5_cls.txt; cat gpurun_out/wc5_cls.txt | head -40
timeout -k 10 600 python -u -m pytest tests/test_device_schedule.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/h_tests.log 2>&1 || { tail -30 gpurun_out/h_tests.log; exit 1; }
tail -1 gpurun_out/h_tests.log
TAG=r04_g bash tools/profile.sh > gpurun_out/profile_g.log 2>&1 || { tail -10 gpurun_out/profile_g.log; exit 1; }
grep -A3 '"lean_kernel_bytes_per_pass"' gpurun_out/prof_r04_g/summary.json
