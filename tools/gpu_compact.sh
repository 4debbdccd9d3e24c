#!/bin/bash
# Compact-boundary + persistence GPU tests, then the bench's host-path legs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
(nproc; cat /sys/fs/cgroup/cpu.max 2>&1; python -c "import os; print(len(os.sched_getaffinity(0)))") > $OUT/cpuinfo.txt
timeout -k 10 400 python -u -m pytest tests/test_compact.py tests/test_persistence.py -m gpu -x -v --timeout 200 \
  --timeout-method thread > $OUT/compact_tests.log 2>&1
rc=$?
tail -12 $OUT/compact_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --cpu-baseline off ${BENCH_ARGS:-} > $OUT/bench_hp.log 2>&1 || { tail -20 $OUT/bench_hp.log; exit 1; }
tail -1 $OUT/bench_hp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); h=d['host_path']; print('compact ms', h.get('ms_per_pass'), 'ext', h.get('ext_records_per_pass'), 'full ms', h.get('full_records', {}).get('ms_per_pass'), h.get('error'))"
cat $OUT/cpuinfo.txt
