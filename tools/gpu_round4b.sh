# The -m gpu suite + smoke, then tools/gpu_cfg_ab.sh (configs vs an older
# build, config kernel trace and counters).
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh || exit $?
bash tools/gpu_cfg_ab.sh
