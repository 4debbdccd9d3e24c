#!/bin/bash
# Wire decode: -m gpu wire tests, then the segment size A/B (GRW_SEG_SHIFT) on
# 512 frames x 8,192 messages and the default 16,384 x 256 workload.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_wire.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/wire_tests.log 2>&1
rc=$?; tail -4 $OUT/wire_tests.log; [ $rc -eq 0 ] || exit $rc
for sh in 13; do
  GRW_SEG_SHIFT=$sh timeout -k 10 120 python -u tools/bench_wire.py --frames 512 --per-frame 8192 --cpu-baseline off > $OUT/wire_8192_s$sh.json 2>$OUT/wire_8192_s$sh.err || exit $?
done
for sh in; do GRW_SEG_SHIFT=$sh timeout -k 10 120 python -u tools/bench_wire.py --cpu-baseline off > $OUT/wire_default_s$sh.json 2>$OUT/wire_default_s$sh.err || exit $?; done
timeout -k 10 120 python -u tools/bench_wire.py --cpu-baseline off > $OUT/wire_default.json 2>$OUT/wire_default.err || exit $?
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/wire_8192_s*.json")) + sorted(glob.glob("gpurun_out/wire_default*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["decode"]["ms"], 3), {k: round(v, 3) for k, v in d["decode"]["phases_ms"].items()})
PY
