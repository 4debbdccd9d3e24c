#!/bin/bash
# Wire codec on the GPU box: -m gpu tests of tests/test_wire.py, the codec bench,
# and a rocprofv3 kernel trace of the bench. Each GPU step has its own limit and
# a crash/abort/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_wire.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/wire_tests.log 2>&1
rc=$?; tail -15 $OUT/wire_tests.log; [ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/bench_wire.py ${WIRE_ARGS:-} > $OUT/wire_bench.json 2> $OUT/wire_bench.err
rc=$?; tail -c 1500 $OUT/wire_bench.json; tail -3 $OUT/wire_bench.err; [ $rc -eq 0 ] || exit $rc
if [ "${PROFILE:-1}" = 1 ]; then
  R=$PWD
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$OUT/prof_wire/trace -o wire -- python3 $R/tools/bench_wire.py --reps 5 --cpu-baseline off > $R/$OUT/prof_wire.log 2>&1 )
  rc=$?; tail -2 $OUT/prof_wire.log; [ $rc -eq 0 ] || exit $rc
  cat $OUT/prof_wire/trace/*kernel_stats.csv | cut -c1-160
fi
echo done
