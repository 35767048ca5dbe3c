#!/bin/bash
# Split-form own-row assignment: the planner's sampler-SIMD weight
# (LPCNET_MF_SIMD_W, tenths; mfw_split_tables default 25) for the skewed
# model at $BS streams, alternating the values in $WS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for w in ${WS:-25 40 60 25 40 60}; do
  LPCNET_MF_SIMD_W=$w timeout -k 10 200 python tools/skew_tput.py ${BS:-8192} > gpurun_out/simdw_$w.log 2>&1 || { echo "w $w rc=$?"; tail -3 gpurun_out/simdw_$w.log; exit 1; }
  echo "w=$w: $(tail -1 gpurun_out/simdw_$w.log | python3 -c 'import sys,json; l=sys.stdin.read().split(" ",1)[1]; d=json.loads(l); print(round(d["skewed"]["samples_per_s"]/1e6,1), "M skewed,", round(d["default"]["samples_per_s"]/1e6,1), "M default")')"
done
