# the exchange's GPU tests, then the one-rank RCCL rehearsal at 1M x 3 traced (one bank, two banks)
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out || exit 1
bash tools/gpu.sh "tests@xch:TESTS=tests/test_pipeline_rccl.py+tests/test_pipeline_world2.py+tests/test_gpu.py::test_cx_pack_unpack+tests/test_gpu.py::test_spread_cold_fields_by_side_buffer+tests/test_gpu.py::test_pipeline_spread_banks" "trace@x1b:GR_BENCH_COLLECTIVE=1,BENCH_ARGS=--placement+spread+--banks+1+--steps+20+--warmup+5+--cpu-baseline+off+--host-path+off" "trace@x2b:GR_BENCH_COLLECTIVE=1,BENCH_ARGS=--placement+spread+--banks+2+--steps+20+--warmup+5+--cpu-baseline+off+--host-path+off" || exit $?
python tools/trace_db.py gpurun_out/trace_x1b --match "" > gpurun_out/trace_x1b.txt 2>&1; head -12 gpurun_out/trace_x1b.txt
python tools/trace_db.py gpurun_out/trace_x2b --match "" > gpurun_out/trace_x2b.txt 2>&1; head -12 gpurun_out/trace_x2b.txt
