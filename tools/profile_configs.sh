#!/bin/bash
# rocprofv3 evidence for BASELINE configs 2, 3 and 5 (tools/bench_configs.py) on
# the GPU box: a kernel trace of every config, then FETCH_SIZE / WRITE_SIZE / SQ
# passes of the configs named in PMC_ONLY (default 3,5), each in its own run with
# its own hard time limit; any failure stops the script.
#   TAG=r03_c bash tools/profile_configs.sh
set -eu
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r03}"
O=$R/gpurun_out/cfgprof_$TAG
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
CFG="$R/tools/bench_configs.py --passes ${PASSES:-10} --warmup 3"
KRE="gr_fast|gr_roles|gr_step|gr_steady|gr_tick|gr_small"
echo "[1] configs + kernel trace"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o cfg -- python3 $CFG --only ${ONLY:-2,3,5} > $O/configs.json 2> $O/trace.log
for c in $(echo ${PMC_ONLY:-3,5} | tr , ' '); do
  echo "[2] config $c FETCH_SIZE"
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -f csv -d $O/fetch$c -o cfg -- python3 $CFG --only $c > $O/fetch$c.log 2>&1
  echo "[3] config $c WRITE_SIZE"
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -f csv -d $O/write$c -o cfg -- python3 $CFG --only $c > $O/write$c.log 2>&1
  echo "[4] config $c SQ"
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --kernel-include-regex "$KRE" -f csv -d $O/sq$c -o cfg -- python3 $CFG --only $c > $O/sq$c.log 2>&1
done
echo "[5] summary"
python3 $R/tools/cfg_prof_summary.py $O > $O/summary.json
cat $O/summary.json
