# exchange GPU tests + the one-rank RCCL rehearsal traced, then the config-3 A/B
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out || exit 1
bash tools/session_exchange.sh || exit $?
bash tools/session_ab_c3.sh || exit $?
