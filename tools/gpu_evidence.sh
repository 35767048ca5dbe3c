#!/bin/bash
# Round evidence in one gpurun call: GPU parity tests, smoke, rocprofv3 kernel
# trace + PMC passes (summarised on the box so the bench line carries the
# measured traffic of this build), bench (with CPU baseline), phase stamps,
# batch-1 traces.  Stops at the first failing GPU step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke rc=$?"; exit 1; }
tail -1 gpurun_out/smoke.log
bash tools/gpu_profile.sh || exit 1
python3 tools/pmc_summary.py gpurun_out > gpurun_out/pmc_summary.log 2>&1 || { echo "pmc summary failed"; exit 1; }
python3 tools/trace_summary.py gpurun_out/prof/run_kernel_trace.csv gpurun_out/trace_summary.json > /dev/null 2>&1 || echo "trace summary: no csv"
timeout -k 10 300 python bench.py --cpu-seconds 10 > gpurun_out/bench.log 2>&1 || { echo "bench rc=$?"; exit 1; }
tail -c 600 gpurun_out/bench.log; echo
timeout -k 10 120 python tools/phase_profile.py 4,5 > gpurun_out/phase.log 2>&1 || { echo "phase rc=$?"; exit 1; }
bash tools/gpu_trace_b1.sh > gpurun_out/trace_b1.log 2>&1 || { echo "b1 trace failed"; exit 1; }
echo "evidence done"
