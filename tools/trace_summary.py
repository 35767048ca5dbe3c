#!/usr/bin/env python3
"""Per-kernel launch durations from a rocprofv3 --kernel-trace CSV, with the
silent launches (the first FEATURES_DELAY frames, which return at once)
separated, so the average is comparable with bench.py's event-timed
avg_launch_ms, per kernel and grid size; mean_us_top averages the longest
launches only (the K-frame multi-frame launches of the timed and preheat
calls); median_us_long / mean_us_long the longest length class without
its outliers, the figures to compare with the bench line's avg_launch_ms.  Usage: trace_summary.py <run_kernel_trace.csv> [out.json]"""
import csv
import json
import sys
from collections import defaultdict


def main(path, out=None):
    d = defaultdict(list)
    spans = []
    for r in csv.DictReader(open(path)):
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        # one entry per (kernel, grid): the same kernel at two batch sizes
        # (mf_kernel<1> at 1 and 256 streams) are two populations
        g = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
        d[f'{r["Kernel_Name"]} [grid {g}]'].append((t1 - t0) / 1e3)
        spans.append((t0, t1))
    res = {}
    for k, v in d.items():
        full = [x for x in v if x > 0.2 * max(v)]  # silent launches return at once
        # the longest launches: the timed K-frame multi-frame launches (the
        # bench's preheat calls run K frames too); shorter multi-frame
        # launches (a first call's K - FEATURES_DELAY frames) fall below 0.95
        top = [x for x in v if x >= 0.95 * max(v)]
        # the longest population by length class: launches within 10 % of
        # the median of the upper half (a few slow outliers no longer set
        # the top class by themselves), and its median -- the figure to
        # compare with the bench line's avg_launch_ms
        upper = sorted(full)[len(full) // 2:] if full else []
        ref = upper[len(upper) // 2] if upper else 0.0
        cls = sorted(x for x in full if abs(x - ref) <= 0.1 * ref)
        res[k] = {"launches": len(v), "mean_us_all": sum(v) / len(v),
                  "launches_non_silent": len(full), "mean_us_non_silent": sum(full) / len(full) if full else None,
                  "launches_top": len(top), "mean_us_top": sum(top) / len(top),
                  "launches_long": len(cls), "median_us_long": cls[len(cls) // 2] if cls else None,
                  "mean_us_long": sum(cls) / len(cls) if cls else None,
                  "min_us": min(v), "max_us": max(v)}
    # idle time of the device between consecutive kernels (host / launch gaps)
    spans.sort()
    gaps = [(b[0] - a[1]) / 1e3 for a, b in zip(spans, spans[1:]) if b[0] > a[1]]
    if gaps:
        gaps.sort()
        res["_gaps_between_kernels_us"] = {"count": len(gaps), "median": gaps[len(gaps) // 2],
                                           "mean": sum(gaps) / len(gaps), "max": gaps[-1]}
    s = json.dumps(res, indent=1)
    print(s)
    if out:
        open(out, "w").write(s)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
