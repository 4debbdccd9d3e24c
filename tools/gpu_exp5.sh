# General-lane A/B builds on config 5 (wave clocks): default, no preload (np),
# full-record message reads (rec), both (nprec).
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in default np rec nprec; do
  if [ $v = default ]; then unset GPURAFT_LIB; else export GPURAFT_LIB=$GRAFT_REPO_ROOT/dragonboat_amd/_build/ab/libgpuraft_$v.so; fi
  GR_WAVE_CLOCK=gpurun_out/wc5_$v.bin timeout -k 10 300 python -u tools/bench_configs.py --passes 10 --only 5 > gpurun_out/exp_c5_$v.json 2> gpurun_out/exp_c5_$v.err || { tail -5 gpurun_out/exp_c5_$v.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/exp_c5_$v.json'):
    d=json.loads(l); print('$v', d['config'][:12], '%.1f us' % (d['device_ms_per_pass']*1e3), 'fast %.1f gen %.1f bailed %d' % (d['fast_ms']*1e3, d['general_ms']*1e3, d['bailed_lanes_per_pass']))
"
  python tools/wave_clock.py gpurun_out/wc5_$v.bin > gpurun_out/wc5_$v.txt; sed -n 3,4p gpurun_out/wc5_$v.txt; grep phase gpurun_out/wc5_$v.txt || true
done
