#!/bin/bash
# tools/gpu.sh — one GPU session as a list of steps, each under its own time
# limit. A crash, abort or timeout (any status other than 0/1) ends the session;
# test failures (status 1) are reported and the session goes on.
#
#   gpurun -- bash tools/gpu.sh STEP [STEP ...]
#
# STEP = KIND[@TAG][:VAR=V,VAR=V...]   (the VARs are set for that step only; a
#        '+' in a value stands for a space: BENCH_ARGS=--groups+2000000)
#   warm              import torch and touch the device (first import is slow)
#   tests             python -m pytest tests -m gpu ($TESTS selects files/-k)
#   bench             bench.py $BENCH_ARGS        -> gpurun_out/bench_TAG.log
#   configs           tools/bench_configs.py $CFG_ARGS -> gpurun_out/cfg_TAG.json
#   trace             rocprofv3 --kernel-trace --stats of bench.py -> gpurun_out/trace_TAG/
#   cfgtrace          the same over tools/bench_configs.py $CFG_ARGS
#   profile           tools/profile.sh (trace + calibrated PMC passes), TAG=...
#   cfgprofile        tools/profile_configs.sh (configs 2, 3, 5 traced; PMC of 3, 5), TAG=...
#   rehearse          bench.py at N = 2 on one GPU over gloo (torch.distributed.run) -> rehearse_TAG.log
#   tickclock         config 3 with GR_WAVE_CLOCK: the tick kernel's wave phases
#   genclock          config 5 with GR_WAVE_CLOCK: the general kernel's wave phases
#   wirepath          tools/bench_wire_path.py at 1M x 3, full and compact outboxes
#   smoke             __graft_entry__.smoke()
# Defaults: BENCH_ARGS="--steps 20 --warmup 5 --cpu-baseline off --host-path off".
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
R=$PWD
: "${BENCH_ARGS:=--steps 20 --warmup 5 --cpu-baseline off --host-path off}"
: "${CFG_ARGS:=--passes 10}"
: "${TESTS:=tests}"

fatal() {  # $1 status, $2 step
  case "$1" in
    0) return 0 ;;
    1) echo "[$2] status 1 (failures), continuing" ; return 0 ;;
    *) echo "[$2] fatal status $1; stopping"; exit "$1" ;;
  esac
}

run_step() {
  local spec="$1" kind tag envs
  kind="${spec%%[@:]*}"
  tag="x"
  [[ "$spec" == *@* ]] && { tag="${spec#*@}"; tag="${tag%%:*}"; }
  envs=""
  [[ "$spec" == *:* ]] && envs="${spec#*:}"
  local -a ev=()
  if [ -n "$envs" ]; then IFS=',' read -r -a ev <<< "$envs"; fi
  local i
  for i in "${!ev[@]}"; do ev[$i]="${ev[$i]//+/ }"; done
  echo "== $kind tag=$tag env=${envs:-none}"
  # the step's variables also reach this script's own expansions ($BENCH_ARGS ...)
  local BENCH_ARGS="$BENCH_ARGS" CFG_ARGS="$CFG_ARGS" TESTS="$TESTS"
  for i in "${!ev[@]}"; do
    case "${ev[$i]}" in BENCH_ARGS=*|CFG_ARGS=*|TESTS=*) eval "${ev[$i]%%=*}=\"\${ev[$i]#*=}\"" ;; esac
  done
  local rc=0
  case "$kind" in
    warm)
      env "${ev[@]}" timeout -k 10 300 python -c "import torch; print(torch.cuda.get_device_name(0))" \
        > $OUT/warm.log 2>&1; rc=$?; tail -1 $OUT/warm.log ;;
    tests)
      env "${ev[@]}" timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 240 \
        --timeout-method thread --durations 15 > $OUT/tests_$tag.log 2>&1; rc=$?; tail -3 $OUT/tests_$tag.log ;;
    bench)
      env "${ev[@]}" timeout -k 10 400 python -u bench.py $BENCH_ARGS > $OUT/bench_$tag.log 2>&1; rc=$?
      python - "$OUT/bench_$tag.log" <<'EOF'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); r = d.get("roofline", {})
        print("ms_per_step %.4f  kernel_ms %.4f  general_ms %.4f  value %.3g" %
              (d["ms_per_step"], r.get("kernel_ms", 0), r.get("general_kernel_ms", 0), d["value"]))
EOF
      ;;
    configs)
      env "${ev[@]}" timeout -k 10 600 python -u tools/bench_configs.py $CFG_ARGS > $OUT/cfg_$tag.json \
        2> $OUT/cfg_$tag.err; rc=$?; tail -2 $OUT/cfg_$tag.err ;;
    trace)
      ( cd /tmp && export TMPDIR=/tmp && env "${ev[@]}" timeout -k 10 400 rocprofv3 --kernel-trace --stats \
          -d $R/$OUT/trace_$tag -o t -- python3 $R/bench.py $BENCH_ARGS > $R/$OUT/trace_$tag.log 2>&1 ); rc=$? ;;
    cfgtrace)
      ( cd /tmp && export TMPDIR=/tmp && env "${ev[@]}" timeout -k 10 600 rocprofv3 --kernel-trace --stats \
          -d $R/$OUT/cfgtrace_$tag -o t -- python3 $R/tools/bench_configs.py $CFG_ARGS \
          > $R/$OUT/cfgtrace_$tag.log 2>&1 ); rc=$? ;;
    profile)
      env "${ev[@]}" TAG=$tag timeout -k 10 900 bash tools/profile.sh > $OUT/profile_$tag.log 2>&1; rc=$?
      tail -3 $OUT/profile_$tag.log ;;
    cfgprofile)
      env "${ev[@]}" TAG=$tag timeout -k 10 900 bash tools/profile_configs.sh > $OUT/cfgprofile_$tag.log 2>&1; rc=$?
      tail -3 $OUT/cfgprofile_$tag.log ;;
    rehearse)  # bench.py's N > 1 script at N = 2 on one GPU, collectives over gloo
      env "${ev[@]}" GR_BENCH_BACKEND=gloo GR_BENCH_ONE_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run \
        --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 \
        $BENCH_ARGS > $OUT/rehearse_$tag.log 2>&1; rc=$?
      grep '^{' $OUT/rehearse_$tag.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=2 ms_per_step %.4f exchange_bytes_per_pass %s heavy %s value %.3g' % (d['ms_per_step'], d.get('exchange_bytes_per_pass'), d.get('exchange_bytes_heavy_pass'), d['value']))" ;;
    tickclock)  # config 3's tick-kernel wave phases (GR_WAVE_CLOCK, tools/tick_clock.py)
      env "${ev[@]}" GR_WAVE_CLOCK=$OUT/wclk_$tag.bin timeout -k 10 300 python -u tools/bench_configs.py --only 3 \
        --passes 6 > $OUT/tickclock_$tag.json 2> $OUT/tickclock_$tag.err; rc=$?
      [ $rc -eq 0 ] && python tools/tick_clock.py $OUT/wclk_$tag.bin | tee $OUT/tickclock_$tag.txt ;;
    genclock)  # config 5's general-kernel wave phases (GR_WAVE_CLOCK, tools/wave_clock.py)
      env "${ev[@]}" GR_WAVE_CLOCK=$OUT/wc5_$tag.bin timeout -k 10 300 python -u tools/bench_configs.py --only 5 \
        --passes 6 > $OUT/genclock_$tag.json 2> $OUT/genclock_$tag.err; rc=$?
      [ $rc -eq 0 ] && python tools/wave_clock.py $OUT/wc5_$tag.bin | tee $OUT/genclock_$tag.txt ;;
    wirepath)  # the 1M x 3 wire path (frames in, tools/bench_wire_path.py), full and compact outboxes
      env "${ev[@]}" timeout -k 10 400 python -u tools/bench_wire_path.py > $OUT/wirepath_$tag.json 2> $OUT/wirepath_$tag.err \
        && env "${ev[@]}" timeout -k 10 400 python -u tools/bench_wire_path.py --compact > $OUT/wirepath_${tag}_compact.json \
        2>> $OUT/wirepath_$tag.err; rc=$?; tail -c 600 $OUT/wirepath_${tag}_compact.json ;;
    smoke)
      env "${ev[@]}" timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
        > $OUT/smoke.log 2>&1; rc=$?; tail -1 $OUT/smoke.log ;;
    *) echo "unknown step $kind"; exit 2 ;;
  esac
  fatal $rc "$kind@$tag"
}

for s in "$@"; do run_step "$s"; done
echo "session done"
