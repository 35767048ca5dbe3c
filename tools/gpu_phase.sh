#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python tools/phase_profile.py > gpurun_out/phase.log 2>&1; rc=$?
cat gpurun_out/phase.log; exit $rc
