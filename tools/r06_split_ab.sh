#!/bin/bash
# Wide split form: parity tests, then skewed throughput (default library and
# the listed variants) and stamped per-wave phases of the skewed model.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "wide" > gpurun_out/split_pytest.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/split_pytest.log; exit 1; }
tail -1 gpurun_out/split_pytest.log
for v in default ${VARIANTS-hlow}; do
  if [ $v = default ]; then unset LPCNET_LIB_VARIANT; else export LPCNET_LIB_VARIANT=$v; fi
  timeout -k 10 200 python tools/skew_tput.py ${BS:-8192} > gpurun_out/skew_$v.log 2>&1 || { echo "skew $v rc=$?"; tail -3 gpurun_out/skew_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/skew_$v.log)"
done
unset LPCNET_LIB_VARIANT
for v in ${STAMPED:-mfwst mfwsth}; do
  PROBE_SKEWED=1 timeout -k 10 120 python tools/mfw_probe.py 8192 4 LPCNET_LIB_VARIANT=$v > gpurun_out/st_$v.log 2>&1 || { echo "st $v rc=$?"; exit 1; }
  echo "== $v"; grep -E "mfw wave [0-9]+ [ERS]:|kernel" gpurun_out/st_$v.log | sort -t' ' -k3 -n
done
