#!/bin/bash
# Skewed-model throughput per forced split plan (LPCNET_MF_CAPS="Tz,Fz,Th,Fh"),
# alternating rounds, one line per run: tools/skew_tput.py at $TB streams.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in ${CAPS:-auto}; do
    if [ "$c" = auto ]; then unset LPCNET_MF_CAPS; else export LPCNET_MF_CAPS=$c; fi
    timeout -k 10 150 python tools/skew_tput.py ${TB:-1024} > gpurun_out/caps_$c.log 2>&1 || { echo "caps $c rc=$?"; tail -5 gpurun_out/caps_$c.log; exit 1; }
    echo "r$r caps=$c $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/caps_$c.log').read().split(' ',1)[1].splitlines()[0]); print(round(d['skewed']['samples_per_s']/1e6,1), round(d['default']['samples_per_s']/1e6,1), round(d['skewed_over_default'],3))")"
  done
done
