# final evidence, part 1: the whole GPU test suite, smoke(), and the headline's trace + calibrated PMC
# (tools/profile.sh: its pmc_latest.json is installed under profiles/ before part 2)
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out || exit 1
bash tools/gpu.sh warm "tests@final" smoke "profile@r06_final" || exit $?
