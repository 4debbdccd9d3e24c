# A/B on config 3 (100k x 5): the current library against a variant (GPURAFT_LIB), interleaved
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out || exit 1
V=$PWD/dragonboat_amd/_build/libgpuraft_tick.so
bash tools/gpu.sh warm "configs@c3a1:CFG_ARGS=--only+3+--passes+20" "configs@c3b1:GPURAFT_LIB=$V,CFG_ARGS=--only+3+--passes+20" "configs@c3b2:GPURAFT_LIB=$V,CFG_ARGS=--only+3+--passes+20" "configs@c3a2:CFG_ARGS=--only+3+--passes+20" || exit $?
for t in c3a1 c3b1 c3b2 c3a2; do python -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/cfg_$t.json') if l.startswith('{')][-1]; print('$t', round(d['device_ms_per_pass']*1e3,1), 'us', round(d['fast_ms']*1e3,1), round(d['general_ms']*1e3,1))"; done
