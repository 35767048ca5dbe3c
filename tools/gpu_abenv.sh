#!/bin/bash
# Alternating A/B of environment settings at one batch size:
#   ENVS="base LPCNET_NO_MULTIFRAME=1" B=1024 ROUNDS=3 tools/gpu_abenv.sh
# "base" = no extra variable.  Prints value and sample-kernel ms per frame.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B=${B:-1024}; ROUNDS=${ROUNDS:-3}; STEPS=${STEPS:-20}; TIMERS=${TIMERS:-1}
for i in $(seq 1 $ROUNDS); do
  for e in $ENVS; do
    tag=$(echo "$e" | tr -c 'A-Za-z0-9_\n' '_')
    if [ "$e" = base ]; then envs=(); else envs=("$e"); fi
    env "${envs[@]}" timeout -k 10 150 python bench.py --streams $B --steps $STEPS --no-cpu --no-batch1 --no-latency --timers $TIMERS > gpurun_out/abe_${tag}_$i.log 2>&1 || { echo "bench $e $i rc=$?"; tail -5 gpurun_out/abe_${tag}_$i.log; exit 1; }
    python3 - gpurun_out/abe_${tag}_$i.log "$e" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("%-28s value %7.4gM step %.4f ms kernel/frame %.4f ms frames/launch %.1f" % (sys.argv[2], d["value"] / 1e6, d["ms_per_step"], r["ms_per_frame"], r["frames_per_launch"]))
PY
  done
done
