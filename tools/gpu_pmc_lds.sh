#!/bin/bash
# One PMC pass of LDS counters over the B=1024 bench (sample kernel bank
# conflicts vs LDS activity), summarised per kernel.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
CTR=${CTR:-"SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"}
timeout -s KILL 90 rocprofv3 --pmc $CTR -d "$R/gpurun_out/pmc_lds" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --streams ${B:-1024} --no-cpu --no-batch1 --no-latency > "$R/gpurun_out/pmc_lds.log" 2>&1 || { echo "pmc rc=$?"; tail -5 "$R/gpurun_out/pmc_lds.log"; exit 1; }
cd "$R"
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/pmc_lds/**/run_counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    print(k, {c: round(v / max(1, n[(k, c)])) for c, v in d.items()})
PY
