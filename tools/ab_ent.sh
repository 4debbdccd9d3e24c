#!/bin/bash
# Entry pass A/B (GRW_ENT_STAGE) and a kernel trace of the wire bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
for st in 1; do
  GRW_ENT_STAGE=$st timeout -k 10 120 python -u tools/bench_wire.py --cpu-baseline off > $OUT/wire_default_st$st.json 2>$OUT/wire_default_st$st.err || exit $?
done
R=$PWD
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/$OUT/prof_wire_f/trace -o wire -- python3 $R/tools/bench_wire.py --reps 5 --cpu-baseline off > $R/$OUT/prof_wire_f.log 2>&1 ) || exit $?
python3 - <<'PY'
import json, glob, csv
for f in sorted(glob.glob("gpurun_out/wire_default_st*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["decode"]["ms"], 3), {k: round(v, 3) for k, v in d["decode"]["phases_ms"].items()})
for f in glob.glob("gpurun_out/prof_wire_f/trace/*kernel_stats.csv"):
    for row in csv.DictReader(open(f)):
        print(row["Name"][:60], row["Calls"], round(float(row["AverageNs"]) / 1e3, 1), "us")
PY
