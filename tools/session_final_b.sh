# final evidence, part 2: configs 2/3/5 traced with PMC (tools/profile_configs.sh) and timed untraced
# (tools/bench_configs.py), their summary installed under profiles/ (bench.py's line carries it: same
# source digest), then the bench line with the CPU baseline and the host path
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out || exit 1
bash tools/gpu.sh warm "cfgprofile@r06_configs:PMC_ONLY=2+3+5" "configs@final:CFG_ARGS=--passes+10" || exit $?
python tools/configs_summary.py gpurun_out/cfgprof_r06_configs gpurun_out/cfg_final.json > gpurun_out/configs_latest.json || exit 1
cp gpurun_out/configs_latest.json profiles/configs_latest.json || exit 1
bash tools/gpu.sh "bench@final:BENCH_ARGS=--steps+20+--warmup+5" || exit $?
