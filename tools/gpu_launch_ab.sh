# Headline A/B: timed passes launched kernel by kernel vs replayed from the
# library's two-pass HIP graph (bench.py --launch), interleaved, same box.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for i in 1 2; do
  for m in stream graph; do
    timeout -k 10 180 python -u bench.py --launch $m --steps 40 --warmup 5 --cpu-baseline off --host-path off > gpurun_out/ab/launch_${m}_$i.json 2> gpurun_out/ab/launch_${m}_$i.err || { tail -5 gpurun_out/ab/launch_${m}_$i.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/ab/launch_${m}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$m', round(d['ms_per_step'],5), round(d['value']/1e9,3), 'G/s kernel', round(r['kernel_ms'],5), d['launch'][:6])"
  done
done
