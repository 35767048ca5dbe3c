#!/bin/bash
# L2 hit rate of the sample and frame kernels (TCC_HIT / TCC_MISS, one PMC
# pass per batch size): are the 3.5 MB embedding tables of the GRU_A gathers
# served by the XCD's L2 or by the Infinity Cache?
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
for B in ${BATCHES:-1024 1}; do
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum -d "$R/gpurun_out/pmc_l2_$B" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --streams $B --no-cpu --no-batch1 > "$R/gpurun_out/pmc_l2_$B.log" 2>&1 || { echo "pmc l2 B=$B rc=$?"; exit 1; }
  echo "l2 B=$B ok"
done
python3 - "$R/gpurun_out" <<'EOF'
import csv, glob, os, statistics, sys
out = sys.argv[1]
for d in sorted(glob.glob(os.path.join(out, "pmc_l2_*"))):
    if not os.path.isdir(d):
        continue
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    per = {}
    for r in rows:
        k = (r["Kernel_Name"][:60], r["Counter_Name"])
        per.setdefault(k, {}).setdefault(r["Dispatch_Id"], 0.0)
        per[k][r["Dispatch_Id"]] += float(r["Counter_Value"])
    names = sorted({k[0] for k in per})
    for n in names:
        med = {c: statistics.median(per[(n, c)].values()) for (m, c) in per if m == n}
        h, m = med.get("TCC_HIT_sum", 0), med.get("TCC_MISS_sum", 0)
        print(os.path.basename(d), n, {c: int(v) for c, v in med.items()}, "hit %.3f" % (h / max(1, h + m)))
EOF
