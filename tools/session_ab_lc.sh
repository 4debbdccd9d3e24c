# A/B: the shipped library (a) against a variant (b, GPURAFT_LIB), interleaved, on
# configs 5 and 3 and the headline pass
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out || exit 1
V=$PWD/dragonboat_amd/_build/libgpuraft_lc.so
C5="CFG_ARGS=--only+5+--passes+10"
C3="CFG_ARGS=--only+3+--passes+10"
bash tools/gpu.sh warm "configs@c5a1:$C5" "configs@c5b1:GPURAFT_LIB=$V,$C5" "configs@c5b2:GPURAFT_LIB=$V,$C5" "configs@c5a2:$C5" \
  "configs@c3a1:$C3" "configs@c3b1:GPURAFT_LIB=$V,$C3" "bench@ha1" "bench@hb1:GPURAFT_LIB=$V" "bench@hb2:GPURAFT_LIB=$V" "bench@ha2" || exit $?
for t in c5a1 c5b1 c5b2 c5a2 c3a1 c3b1; do python -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/cfg_$t.json') if l.startswith('{')][-1]; print('$t', round(d['device_ms_per_pass']*1e3,1), 'us', round(d['fast_ms']*1e3,1), round(d['general_ms']*1e3,1), 'general lanes', d['general_lanes_per_pass'])"; done
for t in ha1 hb1 hb2 ha2; do python -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/bench_$t.log') if l.startswith('{')][-1]; print('$t', d['ms_per_step'], d['value'])"; done
