#!/bin/bash
# Stamped wide kernel (MFW_STAMPS variant): per-wave work / wait per phase,
# default and skewed models at $B streams.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for m in 0 1; do
  PROBE_SKEWED=$m timeout -k 10 120 python tools/mfw_probe.py ${B:-8192} 4 LPCNET_LIB_VARIANT=mfwst > gpurun_out/mfwst_$m.log 2>&1 || { echo "st $m rc=$?"; tail -3 gpurun_out/mfwst_$m.log; exit 1; }
  echo "== skewed=$m"; grep -E "mfw wave|kernel" gpurun_out/mfwst_$m.log | sort -t' ' -k3 -n
done
