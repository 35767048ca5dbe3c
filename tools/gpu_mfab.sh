#!/bin/bash
# mf_kernel change bring-up: parity subset, phase stamps, then an alternating A/B bench against liblpcnet_mi355x_base.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider \
  -k "edge_cases or large_batch or golden or full_size or preload" > gpurun_out/pytest_mf.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|error" gpurun_out/pytest_mf.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python tools/phase_profile.py 4 nofp32 > gpurun_out/phase_mf.log 2>&1; rc=$?
cat gpurun_out/phase_mf.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh 3
