#!/bin/bash
# mfw_kernel with two vs three groups per workgroup: parity, then same-box A/B against mf2_kernel
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "wide_kernel or live_engine" > gpurun_out/mfwg_pt.log 2>&1; rc=$?; tail -2 gpurun_out/mfwg_pt.log; [ $rc -eq 0 ] || exit $rc
for G in 2 3; do
  LPCNET_MFW_G=$G timeout -k 10 300 python tools/ab_env.py LPCNET_MFW=0,1 1536,2048,3072,8192,24576 20 2 > gpurun_out/mfwg_ab_$G.log 2>&1 || { echo "ab rc=$?"; exit 1; }
  echo "G=$G"; cat gpurun_out/mfwg_ab_$G.log
done
