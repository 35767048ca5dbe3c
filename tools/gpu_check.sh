#!/bin/bash
# One gpurun session: GPU parity tests (optionally a -k selection in $K),
# smoke, then the bench line.  Every GPU step has its own time limit; the
# script stops at the first failing step.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
STEPS=${STEPS:-20}
TAG=${TAG:-run}
if [ -n "$FIRST" ]; then
  # the tests of this change first (fail fast), then the whole suite
  timeout -k 10 ${TEST_TIMEOUT:-780} python -u -m pytest $FIRST -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/pt_first_$TAG.log 2>&1
  rc=$?; echo "pytest(first) rc=$rc"; tail -4 gpurun_out/pt_first_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$NOTEST" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-780} python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pt_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pt_$TAG.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke rc=$?"; exit 1; }
  tail -1 gpurun_out/smoke_$TAG.log
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 420 python -u bench.py --steps $STEPS ${BENCH_ARGS} > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
  tail -c 1500 gpurun_out/bench_$TAG.log; echo
fi
echo "gpu_check done"
