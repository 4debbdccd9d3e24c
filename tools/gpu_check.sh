#!/bin/bash
# One GPU session: warm torch, run the -m gpu tests, the bench, and a rocprofv3
# kernel-trace of the bench. Each GPU step has its own time limit; a crash,
# abort or timeout ends the script (test failures, exit 1, do not).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
stop_if_fatal() {  # $1 = exit status of a GPU step
  case "$1" in
    0|1) return 0 ;;
    *) echo "fatal status $1 in $2; stopping"; exit "$1" ;;
  esac
}
timeout -k 10 240 python -c "import torch; print('cuda', torch.cuda.is_available(), torch.cuda.get_device_name(0))" > $OUT/warm.log 2>&1
stop_if_fatal $? warm
echo "warm ok"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?; tail -5 $OUT/gpu_tests.log; stop_if_fatal $rc tests
fi
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
rc=$?; tail -2 $OUT/bench.log; stop_if_fatal $rc bench
if [ "${PROFILE:-1}" = 1 ]; then
  R=$PWD
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof -o bench -- python3 $R/bench.py --steps 10 --warmup 3 --cpu-baseline off > $R/$OUT/prof.log 2>&1 )
  rc=$?; tail -2 $OUT/prof.log; stop_if_fatal $rc rocprof
fi
echo done
