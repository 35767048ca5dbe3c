#!/bin/bash
# Round evidence in one gpurun call: GPU parity tests, smoke, rocprofv3
# kernel-trace stats of the bench command, separate PMC passes per bench
# configuration (HBM bytes, L2 hit rate, MFMA busy), summarised into
# gpurun_out/pmc_traffic.json (stamped with the source hash bench.py checks),
# then the bench line itself.  Stops at the first failing GPU step.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
STEPS=${STEPS:-20}
timeout -k 10 420 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke rc=$?"; exit 1; }
tail -1 gpurun_out/smoke.log
export TMPDIR=/tmp
cd /tmp
# kernel trace + stats of the bench command (all four configurations; two
# warmup frames = the silent FEATURES_DELAY frames, so every non-silent
# launch of a multi-frame kernel covers the same number of frames)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps $STEPS --warmup 2 --no-cpu --no-latency --no-capacity --no-dropin > "$R/gpurun_out/prof.log" 2>&1 || { echo "rocprof trace rc=$?"; exit 1; }
echo "trace ok"
# PMC passes: one counter group per run (slot limits, MI355X_MICROARCH.md)
# (b8192 / b32768: the wide kernel, mfw_kernel, that carries the capacity
# figures; its LDS bank conflicts and wave states as two more passes)
for cfg in "b1024:--streams 1024" "b256:--streams 256" "b1:--streams 1" "b1_fp32:--streams 1 --variant fp32" "b8192:--streams 8192" "b32768:--streams 32768"; do
  name=${cfg%%:*}; args=${cfg#*:}
  passes=("fetch:FETCH_SIZE" "write:WRITE_SIZE" "l2:TCC_HIT_sum TCC_MISS_sum" "mfma:SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "valu:SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE")
  case $name in b1024|b8192|b32768) passes+=("lds:SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" "waves:SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU");; esac
  for pass in "${passes[@]}"; do
    pn=${pass%%:*}; ctr=${pass#*:}
    timeout -s KILL 120 rocprofv3 --pmc $ctr -d "$R/gpurun_out/pmc_${pn}_${name}" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 2 $args --no-cpu --no-batch1 --no-latency --no-capacity --no-dropin > "$R/gpurun_out/pmc_${pn}_${name}.log" 2>&1 || { echo "pmc $pn $name rc=$?"; exit 1; }
  done
  echo "pmc $name ok"
done
cd "$R"
python3 tools/pmc_summary.py gpurun_out gpurun_out/pmc_traffic.json > gpurun_out/pmc_summary.log 2>&1 || { echo "pmc summary failed"; exit 1; }
f=$(ls gpurun_out/prof/*/run_kernel_trace.csv gpurun_out/prof/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/trace_summary.py "$f" gpurun_out/trace_summary.json > /dev/null 2>&1 || echo "trace summary: no csv"
timeout -k 10 400 python bench.py --gpus 1 --steps $STEPS --warmup 5 > gpurun_out/bench.log 2>&1 || { echo "bench rc=$?"; exit 1; }
tail -c 800 gpurun_out/bench.log; echo
echo "evidence done"
