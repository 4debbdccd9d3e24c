#!/bin/bash
# rocprofv3 kernel + memory-copy trace of the compact host path (tools/host_path_prof.py).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/hostprof_${TAG:-x}
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -f csv -d $O/trace -o hp -- python3 $R/tools/host_path_prof.py > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
tail -2 $O/run.log
