# A/B on config 5 (100k x 3): the current library against a variant (GPURAFT_LIB), interleaved
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out || exit 1
V=$PWD/dragonboat_amd/_build/libgpuraft_early.so
bash tools/gpu.sh warm "configs@c5a1:CFG_ARGS=--only+5+--passes+20" "configs@c5b1:GPURAFT_LIB=$V,CFG_ARGS=--only+5+--passes+20" "configs@c5b2:GPURAFT_LIB=$V,CFG_ARGS=--only+5+--passes+20" "configs@c5a2:CFG_ARGS=--only+5+--passes+20" || exit $?
for t in c5a1 c5b1 c5b2 c5a2; do python -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/cfg_$t.json') if l.startswith('{')][-1]; print('$t', round(d['device_ms_per_pass']*1e3,1), 'us', round(d['fast_ms']*1e3,1), round(d['general_ms']*1e3,1))"; done
