#!/usr/bin/env python3
"""Stamped per-phase critical path (bench.latency) of the default model on
mf_kernel's plain and split forms (LPCNET_MF_FORCE_SPLIT) and of the skewed
model, at the given batch sizes."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import lpcnet_amd as L  # noqa: E402

out = {}
for B in [int(x) for x in sys.argv[1].split(",")]:
    cases = (("default", False, False), ("forced_split", False, True), ("skewed", True, False))
    if len(sys.argv) > 2:
        cases = [c for c in cases if c[0] in sys.argv[2].split(",")]
    for name, skew, force in cases:
        if force:
            os.environ["LPCNET_MF_FORCE_SPLIT"] = "1"
        else:
            os.environ.pop("LPCNET_MF_FORCE_SPLIT", None)
        blob = L.synthetic_model(1, 0, skewed=skew)
        out[f"B{B} {name}"] = bench.latency(L, blob, B, 0.0)
        print(f"B{B} {name}", json.dumps(out[f"B{B} {name}"]["critical_path_cycles"]), out[f"B{B} {name}"]["cycles_per_sample"], flush=True)
        if "gru_a_waves" in out[f"B{B} {name}"]:
            print("   recurrent per wave", [round(v["recurrent"]) for v in out[f"B{B} {name}"]["gru_a_waves"].values()], flush=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "split_latency%s.json" % os.environ.get("LPCNET_LIB_VARIANT", "")), "w"), indent=1)
