#!/usr/bin/env python3
"""Summarise rocprofv3 outputs into profiles/<round>/: kernel stats and the
per-launch HBM traffic of the sample kernel from FETCH_SIZE / WRITE_SIZE.
gfx950 correction (MI355X_MICROARCH.md "HBM"): FETCH_SIZE reads half the bytes
of wide coalesced streaming reads -> doubled; both counters are in KB."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def per_kernel(counter_rows, counter):
    agg = {}
    for r in counter_rows:
        if r.get("Counter_Name") != counter:
            continue
        k = r["Kernel_Name"]
        agg.setdefault(k, []).append(float(r["Counter_Value"]))
    return agg


def main(outdir):
    os.makedirs(outdir, exist_ok=True)
    fetch = per_kernel(rows(os.path.join(ROOT, "gpurun_out/pmc_fetch/**/*counter_collection.csv")), "FETCH_SIZE")
    write = per_kernel(rows(os.path.join(ROOT, "gpurun_out/pmc_write/**/*counter_collection.csv")), "WRITE_SIZE")
    res = {}
    for k in set(fetch) | set(write):
        f = fetch.get(k, [])
        w = write.get(k, [])
        # drop the near-empty launches of the silent first frames (FEATURES_DELAY)
        fm = sorted(f)[len(f) // 2] if f else None
        wm = sorted(w)[len(w) // 2] if w else None
        res[k] = {"launches": len(f), "fetch_kb_median": fm, "write_kb_median": wm,
                  "hbm_bytes_per_launch_corrected": (2 * fm * 1024 if fm is not None else 0) + (wm * 1024 if wm is not None else 0)}
    # MFMA utilisation: busy cycles of all SIMDs over (elapsed cycles x 1024
    # SIMDs); elapsed = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs)
    mf = rows(os.path.join(ROOT, "gpurun_out/pmc_mfma/**/*counter_collection.csv"))
    busy, gui, sqb = per_kernel(mf, "SQ_VALU_MFMA_BUSY_CYCLES"), per_kernel(mf, "GRBM_GUI_ACTIVE"), per_kernel(mf, "SQ_BUSY_CYCLES")
    for k in set(busy) & set(gui):
        b, g = sorted(busy[k]), sorted(gui[k])
        bm, gm = b[len(b) // 2], g[len(g) // 2]
        res.setdefault(k, {})
        res[k].update({"mfma_busy_cycles_median": bm, "grbm_gui_active_median": gm,
                       "sq_busy_cycles_median": sorted(sqb.get(k, [0]))[len(sqb.get(k, [0])) // 2],
                       "mfma_util": bm / max(1.0, gm / 8 * 1024)})
    json.dump(res, open(os.path.join(outdir, "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r01"))
