set -u
cd "${GRAFT_REPO_ROOT}"
bash tools/gpu_tests.sh || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || exit $?
cat gpurun_out/bench_final.json
TAG=r03_h bash tools/profile.sh > gpurun_out/profile_h.log 2>&1 || exit $?
TAG=r03_g ONLY=2,3,5 PMC_ONLY=" " bash tools/profile_configs.sh || exit $?
timeout -k 10 200 python tools/bench_wire_path.py --groups 1000000 --passes 3 > gpurun_out/wire_full.json || exit $?
timeout -k 10 200 python tools/bench_wire_path.py --groups 1000000 --passes 3 --compact > gpurun_out/wire_compact.json || exit $?
cat gpurun_out/wire_full.json gpurun_out/wire_compact.json
