#!/bin/bash
# Round evidence in one gpurun call: GPU parity tests, smoke, bench (with CPU
# baseline), rocprofv3 kernel stats + PMC passes, phase stamps.  Stops at the
# first failing GPU step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke rc=$?"; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --cpu-seconds 10 > gpurun_out/bench.log 2>&1 || { echo "bench rc=$?"; exit 1; }
tail -c 600 gpurun_out/bench.log; echo
bash tools/gpu_profile.sh || exit 1
timeout -k 10 120 python tools/phase_profile.py 4 > gpurun_out/phase.log 2>&1 || { echo "phase rc=$?"; exit 1; }
echo "evidence done"
