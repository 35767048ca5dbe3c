#!/bin/bash
# Copy one gpu_evidence.sh run's summaries from gpurun_out/ into profiles/<round>/
# (tracked): pmc_traffic.json (the file bench.py reads, stamped with the source
# hash), tagged copies of the bench line, kernel-trace stats and summaries.
# Usage: tools/save_evidence.sh <round dir, e.g. profiles/r02> <tag>
set -e
D=$1; T=$2
mkdir -p "$D"
cp gpurun_out/pmc_traffic.json "$D/pmc_traffic.json"
cp gpurun_out/pmc_traffic.json "$D/${T}_pmc_traffic.json"
tail -1 gpurun_out/bench.log > "$D/${T}_bench.json"
cp gpurun_out/trace_summary.json "$D/${T}_trace_summary.json"
f=$(ls gpurun_out/prof/*/run_kernel_stats.csv gpurun_out/prof/run_kernel_stats.csv 2>/dev/null | head -1)
cp "$f" "$D/${T}_kernel_stats.csv"
cp gpurun_out/pytest_gpu.log "$D/${T}_pytest_gpu.log"
[ -f gpurun_out/smoke.log ] && cp gpurun_out/smoke.log "$D/${T}_smoke.log"
echo "saved $T into $D"
