#!/usr/bin/env python3
"""Runs the sample kernel on one model for PMC A/B passes:
`pmc_ab.py default|skewed|forced B F` (LPCNET_MF_FORCE_SPLIT for forced)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import lpcnet_amd as L  # noqa: E402

name, B, F = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
if name == "forced":
    os.environ["LPCNET_MF_FORCE_SPLIT"] = "1"
b = L.LPCNetBatch(B, 0, L.synthetic_model(1, 0, skewed=name == "skewed"))
allf = np.ascontiguousarray(np.stack([L.synthetic_features(s, F)[:, :20] for s in range(B)], 1))
df = b.device_alloc(allf.nbytes)
dp = b.device_alloc(F * B * 160 * 2)
b.h2d(df, allf)
b.synthesize_frames(allf, df, dp, F)
b.sync()
print(name, b.info().kernel_name, flush=True)
