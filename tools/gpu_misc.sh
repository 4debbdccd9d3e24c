#!/bin/bash
# Pipeline tests, host-path SDMA A/B, and a spread bench at N=1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -v -k "pipeline or device_resident" --timeout 200 \
  --timeout-method thread > $OUT/pipe_tests.log 2>&1
rc=$?
tail -6 $OUT/pipe_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python3 tools/host_path_prof.py > $OUT/hp_sdma1.json || exit 1
HSA_ENABLE_SDMA=0 timeout -k 10 200 python3 tools/host_path_prof.py > $OUT/hp_sdma0.json || exit 1
for f in $OUT/hp_sdma*.json; do echo $f; python -c "import json; d=json.load(open('$f')); print(d['ms_per_pass'])"; done
timeout -k 10 300 python -u bench.py --steps 20 --placement spread --cpu-baseline off --host-path off > $OUT/bench_spread.log 2>&1 || { tail -5 $OUT/bench_spread.log; exit 1; }
tail -1 $OUT/bench_spread.log | cut -c1-700
