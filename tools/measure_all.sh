set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/bench_h.log 2>&1 || exit 1
tail -1 gpurun_out/bench_h.log
TAG=r01h bash tools/profile.sh > gpurun_out/profile_h.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_configs.py --passes 12 > gpurun_out/configs.json 2> gpurun_out/configs.err || exit 1
timeout -k 10 300 python -u tools/bench_host_path.py --groups 1000000 --passes 5 > gpurun_out/host_path.json 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --placement spread --steps 20 --cpu-baseline off > gpurun_out/spread.log 2>&1 || exit 1
tail -1 gpurun_out/spread.log | cut -c1-200
echo done
