#!/bin/bash
# One measurement session: -m gpu tests + smoke (tools/gpu_tests.sh), the default
# bench line, and the rocprofv3 trace + PMC passes of tools/profile.sh (TAG).
# Each GPU step is time-limited; a crash, abort or timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  bash tools/gpu_tests.sh || exit $?
fi
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-600
if [ "${PROFILE:-1}" = 1 ]; then
  TAG=${TAG:-r02} bash tools/profile.sh > $OUT/profile.log 2>&1 || { tail -20 $OUT/profile.log; exit 1; }
  tail -40 $OUT/profile.log | grep -E "hbm_bytes|AverageNs|gr_fast" | head -10
fi
echo done
