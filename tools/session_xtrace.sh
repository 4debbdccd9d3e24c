# one-rank RCCL rehearsal of the spread exchange at 1M x 3, traced: one bank (kernels alone, no overlap), then two
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out || exit 1
bash tools/gpu.sh "trace@x1b:GR_BENCH_COLLECTIVE=1,BENCH_ARGS=--placement+spread+--banks+1+--steps+20+--warmup+5+--cpu-baseline+off+--host-path+off" "trace@x1bd:GR_BENCH_COLLECTIVE=1,GR_BENCH_CODEC=dense,BENCH_ARGS=--placement+spread+--banks+1+--steps+20+--warmup+5+--cpu-baseline+off+--host-path+off" || exit $?
python tools/trace_db.py gpurun_out/trace_x1b --match "" | head -14
python tools/trace_db.py gpurun_out/trace_x1bd --match "" | head -14
