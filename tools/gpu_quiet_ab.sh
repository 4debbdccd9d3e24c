# quiet_step in one load round (this build) vs the previous build (ab/libgpuraft_prev.so):
# configs 3 and 5 at 10 passes, interleaved, then the device-schedule parity tests.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for i in 1 2; do
  for v in prev new; do
    if [ $v = prev ]; then export GPURAFT_LIB=$GRAFT_REPO_ROOT/dragonboat_amd/_build/ab/libgpuraft_prev.so; else unset GPURAFT_LIB; fi
    timeout -k 10 300 python -u tools/bench_configs.py --passes 10 --only 3,5 > gpurun_out/ab/q_$v$i.json 2> gpurun_out/ab/q_$v$i.err || { tail -5 gpurun_out/ab/q_$v$i.err; exit 1; }
    python -c "
import json
for l in open('gpurun_out/ab/q_$v$i.json'):
    d=json.loads(l); print('$v$i', d['config'][:12], '%.1f us' % (d['device_ms_per_pass']*1e3), 'fast %.1f gen %.1f' % (d['fast_ms']*1e3, d['general_ms']*1e3))
"
  done
done
unset GPURAFT_LIB
timeout -k 10 600 python -u -m pytest tests/test_device_schedule.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/q_tests.log 2>&1 || { tail -30 gpurun_out/q_tests.log; exit 1; }
tail -1 gpurun_out/q_tests.log
