#!/bin/bash
# Live tick A/B at $B streams: the C driver (tools/dropin_bench live) and the
# Python loop (tools/live_probe.py host) under each engine setting in $ENVS,
# alternating $ROUNDS times.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
B=${B:-1024}
for k in $(seq 1 ${ROUNDS:-2}); do
  for e in ${ENVS:-base LPCNET_SYNC_POLL=1}; do
    if [ "$e" = base ]; then envs=(); else envs=("$e"); fi
    c=$(env "${envs[@]}" timeout -k 10 60 ./tools/dropin_bench $B 500 live 2>&1) || { echo "c live rc=$? $c"; exit 1; }
    p=$(env "${envs[@]}" timeout -k 10 120 python tools/live_probe.py $B 300 host 2>&1 | tail -1) || { echo "py live rc=$?"; exit 1; }
    echo "$e | C $c | py $p"
  done
done
