# final evidence, part 2: headline trace + calibrated PMC (tools/profile.sh), configs 2/3/5 traced with
# PMC (tools/profile_configs.sh), their summaries installed under profiles/ (so bench.py's line carries
# them: same source digest), then the bench line with the CPU baseline and the host path
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out || exit 1
bash tools/gpu.sh warm "profile@r06_final" "cfgprofile@r06_configs:PMC_ONLY=2+3+5" || exit $?
cp gpurun_out/prof_r06_final/pmc_latest.json profiles/pmc_latest.json || exit 1
python tools/configs_summary.py gpurun_out/cfgprof_r06_configs > gpurun_out/configs_latest.json || exit 1
cp gpurun_out/configs_latest.json profiles/configs_latest.json || exit 1
bash tools/gpu.sh "bench@final:BENCH_ARGS=--steps+20+--warmup+5" || exit $?
