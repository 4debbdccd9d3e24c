#!/bin/bash
# A/B of engine launch options by environment (one build): bench.py once per
# setting, each in its own process under its own time limit; stops at the first
# fatal status. Usage: tools/ab_env.sh "" "GR_ROLES_MERGED=1" "GR_GENERAL_BLOCKS=1" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
i=0
for setting in "$@"; do
  i=$((i+1))
  env $setting timeout -k 10 180 python -u bench.py --steps ${STEPS:-40} --warmup 5 --cpu-baseline off --host-path off ${BENCH_ARGS:-} > gpurun_out/ab/env$i.json 2> gpurun_out/ab/env$i.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "[$setting] failed rc=$rc"; tail -3 gpurun_out/ab/env$i.err; exit $rc; fi
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab/env$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('[$setting]', round(d['ms_per_step'],4), round(r['kernel_ms'],4), round(r['general_kernel_ms'],4), round(r['frac'],3))"
done
