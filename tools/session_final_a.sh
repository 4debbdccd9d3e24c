# final evidence, part 1: the whole GPU test suite and smoke() on the final build
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out || exit 1
bash tools/gpu.sh warm "tests@final" smoke || exit $?
