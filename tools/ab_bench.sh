#!/bin/bash
# A/B: bench.py against alternative builds of libgpuraft.so (GPURAFT_LIB), each
# in its own process under its own time limit; stops at the first fatal status.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for lib in dragonboat_amd/_build/libgpuraft.so "$@"; do
  name=$(basename $lib .so)
  GPURAFT_LIB=$PWD/$lib timeout -k 10 180 python -u bench.py --steps 40 --warmup 5 --cpu-baseline off > gpurun_out/ab/$name.json 2> gpurun_out/ab/$name.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; tail -3 gpurun_out/ab/$name.err; exit $rc; fi
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$name', round(d['ms_per_step'],4), round(r['kernel_ms'],4), round(r['frac'],3))"
done
