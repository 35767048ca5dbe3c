#!/bin/bash
# Two-group kernel bring-up: its parity tests, then phase stamps (modes 6 and 4), then the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider \
  -k "two_group or large_batch or golden" > gpurun_out/pytest_mfp.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|error" gpurun_out/pytest_mfp.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python tools/phase_profile.py 6,4 nofp32 > gpurun_out/phase_mfp.log 2>&1; rc=$?
cat gpurun_out/phase_mfp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --no-cpu > gpurun_out/bench_mfp.log 2>&1 || exit $?
tail -1 gpurun_out/bench_mfp.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.4g'%d['value'], d['roofline']['kernel'], 'ms %.4f'%d['roofline']['avg_launch_ms'], 'frac %.3f'%d['roofline']['frac'], 'b1 %.4g'%d['batch1']['samples_per_s'], 'b256 %.4g'%d['batch256']['samples_per_s'])"
