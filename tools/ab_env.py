#!/usr/bin/env python3
"""Same-box A/B of engine environment switches on the device-resident frame
step: python tools/ab_env.py VAR=a,b B1,B2,... [steps] [rounds] [variant]
(variant int8 / int8_skewed / fp32 / fp32_skewed).  Alternates the settings
round by round (each in a fresh batch) and prints ms per frame step."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import lpcnet_amd as L  # noqa: E402

var, vals = sys.argv[1].split("=")
vals = vals.split(",")
Bs = [int(x) for x in sys.argv[2].split(",")]
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 3
variant = sys.argv[5] if len(sys.argv) > 5 else "int8"
blob = L.synthetic_model(1, 1 if variant.startswith("fp32") else 0, skewed=variant.endswith("skewed"))
res = {}
for B in Bs:
    for r in range(rounds):
        for v in vals:
            os.environ[var] = v
            dt, (k, n, kf, _, _), info, _ = bench.run_batch(L, blob, B, 0, 3, steps, None, 1, 30.0 if r == 0 else 0.0)
            res.setdefault(f"B{B} {var}={v}", []).append((dt / steps * 1e3, k / max(kf, 1), info.kernel_name))
for k, v in res.items():
    ms = sorted(x[0] for x in v)
    print(f"{k}: frame step {ms[len(ms)//2]:.4f} ms (min {ms[0]:.4f}), sample kernel {sorted(x[1] for x in v)[len(v)//2]:.4f} ms/frame, {v[0][2]}")
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", f"ab_{var}.json"), "w"))
