#!/bin/bash
# rocprofv3 evidence for bench.py's dominant kernel (run on the GPU box):
#   1. kernel trace + stats (CSV) of the default bench workload
#   2. separate PMC passes: FETCH_SIZE, WRITE_SIZE, SQ occupancy/stall counters
#   3. the same FETCH/WRITE passes over tools/hbm_calib (known byte counts)
# Every rocprofv3 run has its own hard time limit; any failure stops the script.
set -eu
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r01}"
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
BENCH="$R/bench.py --steps ${STEPS:-10} --warmup 3 --cpu-baseline off ${BENCH_ARGS:-}"
# counter passes: the device-resident passes only (the host-path leg runs other kernels)
BENCH_PMC="$BENCH --host-path off"
KRE="gr_fast|gr_roles|gr_step|gr_steady|gr_tick"
echo "[0] available counters (non-fatal)"
timeout -s KILL 60 rocprofv3 -L > $O/counters_avail.txt 2>&1 || echo "counter list failed"
echo "[1] kernel trace"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o bench -- python3 $BENCH > $O/trace.log 2>&1
echo "[2] FETCH_SIZE"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -f csv -d $O/fetch -o bench -- python3 $BENCH_PMC > $O/fetch.log 2>&1
echo "[3] WRITE_SIZE"
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -f csv -d $O/write -o bench -- python3 $BENCH_PMC > $O/write.log 2>&1
echo "[4] SQ"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --kernel-include-regex "$KRE" -f csv -d $O/sq -o bench -- python3 $BENCH_PMC > $O/sq.log 2>&1
echo "[4b] SQ instruction mix and in-flight vector memory (non-fatal: counter names vary by ROCm)"
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INST_LEVEL_VMEM SQ_WAIT_INST_ANY SQ_WAVES SQ_INSTS_VMEM --kernel-include-regex "$KRE" -f csv -d $O/sq2 -o bench -- python3 $BENCH_PMC > $O/sq2.log 2>&1 || echo "sq2 pass failed (see sq2.log)"
echo "[5] calibration"
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/calib_fetch -o calib -- $R/tools/hbm_calib > $O/calib_fetch.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/calib_write -o calib -- $R/tools/hbm_calib > $O/calib_write.log 2>&1
echo "[6] summary"
python3 $R/tools/prof_summary.py $O > $O/summary.json
cat $O/summary.json
