#!/bin/bash
# The -m gpu suite on the box (each step time-limited; a crash, abort or
# timeout ends the script), then smoke().
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 240 python -c "import torch; print('cuda', torch.cuda.is_available(), torch.cuda.get_device_name(0))" > $OUT/warm.log 2>&1 || exit $?
echo "warm ok"
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=25 ${PYTEST_ARGS:-} > $OUT/gpu_tests.log 2>&1
rc=$?
tail -15 $OUT/gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc2=$?
tail -3 $OUT/smoke.log
exit $(( rc > rc2 ? rc : rc2 ))
