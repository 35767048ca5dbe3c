#!/bin/bash
# GPU parity tests (stop at the first failure), then an alternating A/B of
# library variants (tools/gpu_abn.sh; VARIANTS, B, ROUNDS as there).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
LPCNET_VERBOSE=1 timeout -k 10 60 python bench.py --steps 4 --no-cpu --no-batch1 --no-latency 2>&1 | grep "range bounds" | head -2
bash tools/gpu_abn.sh
