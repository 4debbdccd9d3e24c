# Role-instance grid A/B (env, one build): headline bench and config 5.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
STEPS=40 bash tools/ab_env.sh "" "GR_ROLE_BLOCKS=512" "GR_ROLE_BLOCKS=256" "GR_ROLES_MERGED=1" "GR_ROLES_MERGED=1 GR_ROLE_BLOCKS=512" || exit 1
for setting in "" "GR_ROLE_BLOCKS=512" "GR_ROLE_BLOCKS=256" "GR_ROLES_MERGED=1"; do
  env $setting timeout -k 10 300 python -u tools/bench_configs.py --passes 8 --only 3,5 > gpurun_out/ab/roles_c5.json 2> gpurun_out/ab/roles_c5.err || { tail -5 gpurun_out/ab/roles_c5.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/ab/roles_c5.json'):
    d=json.loads(l); print('[$setting]', d['config'][:12], '%.1f us' % (d['device_ms_per_pass']*1e3), 'fast %.1f gen %.1f' % (d['fast_ms']*1e3, d['general_ms']*1e3))
"
done
