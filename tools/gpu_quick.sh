#!/bin/bash
# Quick GPU iteration: parity tests (stop at first failure), phase stamps of
# the pipelined kernels, short bench.  KERNELS selects the phase-profile modes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python tools/phase_profile.py ${KERNELS:-3,4} nofp32 > gpurun_out/phase.log 2>&1 || { echo "phase rc=$?"; exit 1; }
cat gpurun_out/phase.log
timeout -k 10 200 python bench.py --steps 20 --no-cpu > gpurun_out/bench.log 2>&1 || exit $?
python3 -c "
import json; d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1])
print('value %.4g'%d['value'], d['roofline']['kernel'], 'sample_ms %.3f'%d['roofline']['avg_launch_ms'], 'frame_ms %.3f'%d['frame_kernel_avg_ms'], 'b1 %.4g'%d['batch1']['samples_per_s'], 'b1fp32 %.4g'%d['batch1_fp32']['samples_per_s'])"
