# A/B of launch options (tools/ab_env.sh), then the -m gpu suite and smoke().
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab_env.sh ${AB_SETTINGS:-"A=1" "A=2"} > gpurun_out/ab_env.log 2>&1 || { cat gpurun_out/ab_env.log; exit 1; }
cat gpurun_out/ab_env.log
bash tools/gpu_tests.sh
