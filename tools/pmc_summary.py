#!/usr/bin/env python3
"""Summarise the rocprofv3 PMC passes of tools/gpu_evidence.sh into one JSON
record per bench configuration:

  {"source_sha256": <hash of lpcnet_amd/csrc + Makefile>,
   "configs": {"b1024": {"<kernel>": {...}}, "b256": ..., "b1": ..., "b1_fp32": ...}}

per kernel: median over its non-silent launches of
  hbm_bytes_per_launch   2 x FETCH_SIZE + WRITE_SIZE (KB counters; gfx950:
                         FETCH_SIZE reads half the bytes of wide reads,
                         MI355X_MICROARCH.md "HBM")
  l2_hit                 TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
  mfma_util              SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
and, for the kernel the pass's bench line names, frames_per_launch (from
that line: a multi-frame launch covers several frames) and
hbm_bytes_per_frame.  bench.py reads it back only when source_sha256 matches
the tree it runs from.
Usage: pmc_summary.py <gpurun_out dir> <out.json>"""
import csv
import glob
import hashlib
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def source_sha256(root=ROOT):
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(root, "lpcnet_amd", "csrc", "*"))) + [os.path.join(root, "Makefile")]
    for f in files:
        if os.path.isfile(f):
            h.update(os.path.basename(f).encode())
            h.update(open(f, "rb").read())
    return h.hexdigest()


def counters(d):
    """{kernel: {counter: [per-dispatch values]}} of one pass directory"""
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            per.setdefault(k, {}).setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
            per[k][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: {c: list(v.values()) for c, v in cs.items()} for k, cs in per.items()}


def med_nonsilent(vals):
    """median over launches above 20 % of the largest (drops the silent first frames)"""
    if not vals:
        return None
    top = max(vals)
    keep = [v for v in vals if v >= 0.2 * top] or vals
    return statistics.median(keep)


def bench_line(log):
    """the bench's JSON line in a pass log: rocprofv3 prints its own lines
    after the program's (round 4 read only the last line and so never found
    it -- no frames_per_launch, roofline.traffic per launch of unknown length)"""
    try:
        lines = open(log).read().splitlines()
    except OSError:
        return None
    for ln in reversed(lines):
        ln = ln.strip()
        if ln.startswith("{") and '"roofline"' in ln:
            try:
                return json.loads(ln)
            except ValueError:
                continue
    return None


def kernel_match(short, full):
    """bench's ModelInfo.kernel_name ('mf_kernel<4, 0, false, true>') in a
    rocprofv3 kernel name ('void lpcnet_mi355x::mf_kernel<4, 0, false,
    true>(lpcnet_mi355x::SampleArgs)'), spacing-insensitive"""
    return short.replace(" ", "") in full.replace(" ", "")


def main(outdir, out):
    res = {"source_sha256": source_sha256(), "configs": {}}
    for d in sorted(glob.glob(os.path.join(outdir, "pmc_*_*"))):
        if not os.path.isdir(d):
            continue
        cfg = os.path.basename(d).split("_", 2)[2]  # pmc_<pass>_<config>
        for k, cs in counters(d).items():
            rec = res["configs"].setdefault(cfg, {}).setdefault(k, {})
            for c, vals in cs.items():
                rec[c] = med_nonsilent(vals)
    fpl = {}
    for log in glob.glob(os.path.join(outdir, "pmc_*_*.log")):
        cfg = os.path.basename(log)[:-4].split("_", 2)[2]
        line = bench_line(log)
        if line is not None:
            fpl.setdefault(cfg, {})[line["roofline"]["kernel"]] = float(line["roofline"].get("frames_per_launch", 1.0))
    for cfg, ks in res["configs"].items():
        for k, r in ks.items():
            for name, f in fpl.get(cfg, {}).items():
                if kernel_match(name, k):
                    r["frames_per_launch"] = f
            if "FETCH_SIZE" in r and "WRITE_SIZE" in r:
                r["hbm_bytes_per_launch"] = 2 * r["FETCH_SIZE"] * 1024 + r["WRITE_SIZE"] * 1024
                if "frames_per_launch" in r:
                    r["hbm_bytes_per_frame"] = r["hbm_bytes_per_launch"] / r["frames_per_launch"]
            if "TCC_HIT_sum" in r and "TCC_MISS_sum" in r:
                r["l2_hit"] = r["TCC_HIT_sum"] / max(1.0, r["TCC_HIT_sum"] + r["TCC_MISS_sum"])
            if "SQ_VALU_MFMA_BUSY_CYCLES" in r and "GRBM_GUI_ACTIVE" in r:
                r["mfma_util"] = r["SQ_VALU_MFMA_BUSY_CYCLES"] / max(1.0, r["GRBM_GUI_ACTIVE"] / 8 * 1024)
            # VALU issue: wave64 VALU instructions per launch against the
            # CU's issue peak (4 SIMD-32s, one wave64 instruction per 2
            # cycles each: 2 per CU-cycle, MI355X_MICROARCH.md "Wave
            # scheduling") over the launch's GPU-busy cycles (GRBM_GUI_ACTIVE
            # sums the 8 XCDs); per frame when the launch length is known
            gui = r.get("GRBM_GUI_ACTIVE_valu", r.get("GRBM_GUI_ACTIVE"))
            if "SQ_INSTS_VALU" in r and gui:
                r["valu_insts_per_launch"] = r["SQ_INSTS_VALU"]
                r["valu_issue_frac"] = r["SQ_INSTS_VALU"] / max(1.0, gui / 8 * 256 * 2)
                if "frames_per_launch" in r:
                    r["valu_insts_per_frame"] = r["SQ_INSTS_VALU"] / r["frames_per_launch"]
            # LDS bank conflicts per LDS-busy cycle; wave states per wave-cycle
            if "SQ_LDS_BANK_CONFLICT" in r and r.get("SQ_ACTIVE_INST_LDS"):
                r["lds_bank_conflict_frac"] = r["SQ_LDS_BANK_CONFLICT"] / r["SQ_ACTIVE_INST_LDS"]
            if r.get("SQ_WAVE_CYCLES"):
                wc = r["SQ_WAVE_CYCLES"]
                r["wave_states"] = {k: r[c] / wc for k, c in (("issuing", "SQ_ACTIVE_INST_ANY"),
                                                             ("valu", "SQ_ACTIVE_INST_VALU"),
                                                             ("waiting", "SQ_WAIT_ANY"),
                                                             ("issue_stalled", "SQ_WAIT_INST_ANY")) if c in r}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
