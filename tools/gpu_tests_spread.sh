# The -m gpu suite + smoke, then bench.py local vs spread at N = 1 (1M x 3).
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit $?
AB_SETTINGS="A=1" BENCH_ARGS="--placement spread" bash tools/ab_env.sh "A=spread" > gpurun_out/ab_spread.log 2>&1 || { cat gpurun_out/ab_spread.log; exit 1; }
cat gpurun_out/ab_spread.log
bash tools/ab_env.sh "A=local" >> gpurun_out/ab_spread.log 2>&1 || { cat gpurun_out/ab_spread.log; exit 1; }
tail -1 gpurun_out/ab_spread.log
