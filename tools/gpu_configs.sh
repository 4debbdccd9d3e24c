#!/bin/bash
# GPU tests (full -m gpu suite), then the per-config device-pass bench and the
# host-path legs. Each step time-limited; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != 1 ]; then bash tools/gpu_tests.sh || exit $?; fi
timeout -k 10 300 python -u tools/bench_configs.py --passes 20 > $OUT/configs.json 2> $OUT/configs.err || { tail -5 $OUT/configs.err; exit 1; }
python -c "
import json
for l in open('$OUT/configs.json'):
    d=json.loads(l); print(d['config'][:40], '%.1f us' % (d['device_ms_per_pass']*1e3), 'fast %.1f gen %.1f' % (d['fast_ms']*1e3, d['general_ms']*1e3), 'esc/pass', d['escalations_per_pass'], d['last_pass_escalations'])
"
GR_PHASES=1 timeout -k 10 250 python3 tools/host_path_prof.py > $OUT/hp.log 2>&1 || { tail -5 $OUT/hp.log; exit 1; }
grep -v gr_phases $OUT/hp.log | python -c "
import json,sys
for l in sys.stdin:
    l=l.strip()
    if l.startswith('{'): d=json.loads(l); print('host path P=%d: %.2f ms/pass' % (d['partitions'], d['ms_per_pass']))
"
grep gr_phases $OUT/hp.log | tail -2
