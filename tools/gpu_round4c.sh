# gr_step boundary tests (the counting sort), then tools/gpu_cfg_ab.sh.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_compact.py tests/test_wire_path.py tests/test_wire.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/io_tests.log 2>&1
rc=$?; tail -3 gpurun_out/io_tests.log; [ $rc -le 1 ] || exit $rc
bash tools/gpu_cfg_ab.sh
