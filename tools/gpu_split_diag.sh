#!/bin/bash
# Split-form diagnostics on one box: for each library variant, the stamped
# per-wave critical path (LPCNET_FINE_STAMPS) of the default and skewed
# models at $B, and their throughput at $TB.
#   VARIANTS="base noatom" B=1024 TB=1024,2048 tools/gpu_split_diag.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B=${B:-1024}; TB=${TB:-1024,2048}
for v in $VARIANTS; do
  if [ "$v" = default ]; then unset LPCNET_LIB_VARIANT; else export LPCNET_LIB_VARIANT=$v; fi
  echo "== $v"
  LPCNET_FINE_STAMPS=1 timeout -k 10 120 python tools/split_latency.py $B default,skewed || exit 1
  timeout -k 10 200 python tools/skew_tput.py $TB || exit 1
done
