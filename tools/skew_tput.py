#!/usr/bin/env python3
"""Throughput of the default and the skewed (trained-mask-like) int8 model at
1, 256 and 1024 streams (or the comma list argv[1]) through bench.run_batch (the bench's own timed path),
and the skewed/default ratio: gpurun_out/skew_tput.json."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import lpcnet_amd as L  # noqa: E402

out = {}
for B in ([int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else (1, 256, 1024)):
    row = {}
    for name, skew in (("default", False), ("skewed", True), ("skewed_no_mfw_split", True)):
        # skewed_no_mfw_split: the same model without the wide kernel's split
        # form (LPCNET_NO_MFW_SPLIT=1: mf2_kernel's split form)
        if name == "skewed_no_mfw_split":
            os.environ["LPCNET_NO_MFW_SPLIT"] = "1"
        blob = L.synthetic_model(1, L.VARIANT_INT8, skewed=skew)
        nf = 40
        dt, _, info, _ = bench.run_batch(L, blob, B, 0, 5, nf, None, 0, 100.0)
        os.environ.pop("LPCNET_NO_MFW_SPLIT", None)
        row[name] = {"samples_per_s": B * nf * 160 / dt, "kernel": info.kernel_name}
    row["skewed_over_default"] = row["skewed"]["samples_per_s"] / row["default"]["samples_per_s"]
    out[f"b{B}"] = row
    print(f"b{B}", json.dumps(row), flush=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "skew_tput%s.json" % os.environ.get("LPCNET_LIB_VARIANT", "")), "w"),
          indent=1)
