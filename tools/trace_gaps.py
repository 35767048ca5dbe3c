#!/usr/bin/env python3
"""Dispatch timeline of a rocprofv3 --kernel-trace CSV: per kernel name the
durations, and the idle gap from each dispatch's end to the next one's start
(tools/gpu_gap.sh)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = defaultdict(list)
gaps = defaultdict(list)
for a, b in zip(rows, rows[1:]):
    gaps[(a["Kernel_Name"][:40], b["Kernel_Name"][:40])].append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
for r in rows:
    dur[r["Kernel_Name"][:40]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in dur.items():
    v.sort()
    print("%-42s n=%4d  median %9.2f us  min %9.2f" % (k, len(v), v[len(v) // 2], v[0]))
print("gaps (us):")
for k, v in sorted(gaps.items(), key=lambda kv: -len(kv[1])):
    v.sort()
    print("  %-40s -> %-40s n=%4d median %7.2f min %7.2f max %8.2f" % (k[0], k[1], len(v), v[len(v) // 2], v[0], v[-1]))
