#!/bin/bash
# Skewed (split form) throughput at $BS streams under issue-priority variants
# of mfw_kernel (tools/ab_build.sh libraries named in $VARIANTS), default first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for v in default ${VARIANTS}; do
  if [ $v = default ]; then unset LPCNET_LIB_VARIANT; else export LPCNET_LIB_VARIANT=$v; fi
  timeout -k 10 200 python tools/skew_tput.py ${BS:-8192} > gpurun_out/prio_$v.log 2>&1 || { echo "skew $v rc=$?"; tail -3 gpurun_out/prio_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/prio_$v.log)"
done
