# Config 2 (10k x 3) launch schedules, A/B on one box: the fused small-pass
# kernel (default), the mid-size path (lean FL_ANY kernel + general kernel:
# GR_SMALL_BLOCKS=0), and the split schedule (GR_SMALL_BLOCKS=0
# GR_SPLIT_MIN_LANES=1); events per pass and the library graph replay, then a
# kernel trace of each.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cfg2
for setting in "A=fused" "GR_SMALL_BLOCKS=0" "GR_SMALL_BLOCKS=0 GR_SPLIT_MIN_LANES=1"; do
  tag=$(echo $setting | tr ' =' '__')
  env $setting timeout -k 10 200 python -u tools/bench_configs.py --passes 20 --only 2 > gpurun_out/cfg2/$tag.json 2> gpurun_out/cfg2/$tag.err || { tail -5 gpurun_out/cfg2/$tag.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/cfg2/$tag.json').read().strip().splitlines()[-1])
print('[$setting]', '%.1f us events' % (d['device_ms_per_pass']*1e3), 'graph %.1f us' % (d['graph']['ms_per_pass']*1e3))
"
  R=$PWD
  ( cd /tmp && export TMPDIR=/tmp && env $setting timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/cfg2/prof_$tag -o cfg -- python3 $R/tools/bench_configs.py --passes 20 --only 2 > $R/gpurun_out/cfg2/prof_$tag.log 2>&1 ) || exit 1
  python -c "
import csv,glob
for f in glob.glob('gpurun_out/cfg2/prof_$tag/**/cfg_kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'gr_' in r['Name'] and 'io::' not in r['Name']: print('   ', r['Name'].split('(')[0][:60], r['Calls'], '%.1f' % (float(r['AverageNs'])/1e3), '%.1f' % (float(r['MinNs'])/1e3))
"
done
