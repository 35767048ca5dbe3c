#!/usr/bin/env python3
"""Per-kernel launch durations from a rocprofv3 --kernel-trace CSV, with the
silent launches (the first FEATURES_DELAY frames, which return at once)
separated, so the average is comparable with bench.py's event-timed
avg_launch_ms.  Usage: trace_summary.py <run_kernel_trace.csv> [out.json]"""
import csv
import json
import sys
from collections import defaultdict


def main(path, out=None):
    d = defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    res = {}
    for k, v in d.items():
        full = [x for x in v if x > 50.0]  # us; silent launches take a few us
        res[k] = {"launches": len(v), "mean_us_all": sum(v) / len(v),
                  "launches_non_silent": len(full), "mean_us_non_silent": sum(full) / len(full) if full else None,
                  "min_us": min(v), "max_us": max(v)}
    s = json.dumps(res, indent=1)
    print(s)
    if out:
        open(out, "w").write(s)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
