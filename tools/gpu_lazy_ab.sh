# A/B of the lazy-remote-rows variant (ab/libgpuraft_lazy.so, commit 3881b00's source,
# reverted in the tree): config 5 at 10 passes interleaved with the product build, and
# the device-schedule parity tests on the variant.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for i in 1 2; do
  for v in prod lazy; do
    if [ $v = lazy ]; then export GPURAFT_LIB=$GRAFT_REPO_ROOT/dragonboat_amd/_build/ab/libgpuraft_lazy.so; else unset GPURAFT_LIB; fi
    timeout -k 10 300 python -u tools/bench_configs.py --passes 10 --only 5 > gpurun_out/ab/l_$v$i.json 2> gpurun_out/ab/l_$v$i.err || { tail -5 gpurun_out/ab/l_$v$i.err; exit 1; }
    python -c "
import json
d=json.loads(open('gpurun_out/ab/l_$v$i.json').read().strip().splitlines()[-1]); print('$v$i', '%.1f us' % (d['device_ms_per_pass']*1e3), 'fast %.1f gen %.1f' % (d['fast_ms']*1e3, d['general_ms']*1e3))
"
  done
done
export GPURAFT_LIB=$GRAFT_REPO_ROOT/dragonboat_amd/_build/ab/libgpuraft_lazy.so
timeout -k 10 600 python -u -m pytest tests/test_device_schedule.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/lazy_tests.log 2>&1; rc=$?; tail -1 gpurun_out/lazy_tests.log; exit $rc
