#!/bin/bash
# rocprofv3: kernel-trace stats, then FETCH_SIZE, WRITE_SIZE and the MFMA
# busy cycles in separate passes (PMC slot limits; MI355X_MICROARCH.md).
# Same command and step count as the bench line.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
STEPS=${STEPS:-30}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps $STEPS --no-cpu --no-batch1 > "$R/gpurun_out/prof.log" 2>&1 || { echo "rocprof trace rc=$?"; exit 1; }
echo "trace ok"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_fetch" -o run --output-format csv -- python3 "$R/bench.py" --steps $STEPS --no-cpu --no-batch1 > "$R/gpurun_out/pmc_fetch.log" 2>&1 || { echo "pmc fetch rc=$?"; exit 1; }
echo "fetch ok"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_write" -o run --output-format csv -- python3 "$R/bench.py" --steps $STEPS --no-cpu --no-batch1 > "$R/gpurun_out/pmc_write.log" 2>&1 || { echo "pmc write rc=$?"; exit 1; }
echo "write ok"
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$R/gpurun_out/pmc_mfma" -o run --output-format csv -- python3 "$R/bench.py" --steps $STEPS --no-cpu --no-batch1 > "$R/gpurun_out/pmc_mfma.log" 2>&1 || { echo "pmc mfma rc=$?"; exit 1; }
echo "mfma ok"
