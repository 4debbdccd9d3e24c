#!/bin/bash
# rocprofv3 kernel trace + SQ counters of tools/bench_configs.py (one config at a time).
set -eu
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/profcfg_${ONLY:-3}
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
ARGS="$R/tools/bench_configs.py --only ${ONLY:-3} --passes 6 --warmup 2"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o cfg -- python3 $ARGS > $O/trace.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --kernel-include-regex "gr_fast|gr_step" -f csv -d $O/sq -o cfg -- python3 $ARGS > $O/sq.log 2>&1
python3 - $O <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
for f in glob.glob(o + "/trace/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gr_" in r["Name"]:
            print("stats", r["Name"][:60], r["Calls"], r["AverageNs"])
per = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(o + "/sq/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        per[r["Kernel_Name"][:40]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in per.items():
    print("sq", k, {c: int(x) for c, x in v.items()})
PY
