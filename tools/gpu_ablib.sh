#!/bin/bash
# Same-box A/B of in-tree library variants on the device-resident frame step
# (tools/ab_env.py), alternating variants round by round:
#   VARIANTS="default base" BS=1024,1 ROUNDS=3 [MODEL=int8|int8_skewed|fp32] [K=<pytest -k>] [AB_VAR=ENV=a,b] tools/gpu_ablib.sh
# (AB_VAR: an engine environment switch alternated inside each variant run)
# "default" = liblpcnet_mi355x.so; <name> = liblpcnet_mi355x_<name>.so
# (tools/ab_build.sh).  With K set, the GPU tests matching K run first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "$K" > gpurun_out/pt_ab.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_ab.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in $VARIANTS; do
    if [ "$v" = default ]; then unset LPCNET_LIB_VARIANT; else export LPCNET_LIB_VARIANT=$v; fi
    timeout -k 10 200 python tools/ab_env.py ${AB_VAR:-LPCNET_AB_ROUND=$r} ${BS:-1024} 20 1 ${MODEL:-int8} > gpurun_out/ablib_${v}_$r.log 2>&1 || { echo "ab $v $r rc=$?"; tail -5 gpurun_out/ablib_${v}_$r.log; exit 1; }
    sed "s/^/$v r$r /" gpurun_out/ablib_${v}_$r.log | grep frame
  done
done
