#!/bin/bash
# SQ instruction-mix, FETCH_SIZE and WRITE_SIZE counters of the wire-codec kernels (one PMC pass each).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/pmc_wire
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --kernel-include-regex "decode_msgs|decode_ents|walk_frames|map_ents|size_msgs|write_msgs" -f csv -d $O/sq -o wire -- python3 $R/tools/bench_wire.py --reps 2 --cpu-baseline off > $O/sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "decode_msgs|decode_ents|walk_frames|map_ents|size_msgs|write_msgs" -f csv -d $O/fetch -o wire -- python3 $R/tools/bench_wire.py --reps 2 --cpu-baseline off > $O/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "decode_msgs|decode_ents|walk_frames|map_ents|size_msgs|write_msgs" -f csv -d $O/write -o wire -- python3 $R/tools/bench_wire.py --reps 2 --cpu-baseline off > $O/write.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
import os
O = os.environ.get("O")
PY
for f in $O/sq/*counter_collection.csv $O/fetch/*counter_collection.csv $O/write/*counter_collection.csv; do
  python3 -c "
import csv,sys,collections
d=collections.defaultdict(lambda: collections.defaultdict(float)); n=collections.Counter()
for r in csv.DictReader(open('$f')):
    k=r['Kernel_Name'].split('(')[0]; d[k][r['Counter_Name']]+=float(r['Counter_Value'])
    n[(k,r['Counter_Name'])]+=1
for k,v in d.items():
    print(k, {c: round(x/ max(1,n[(k,c)]) if False else x,1) for c,x in v.items()})
"
done
