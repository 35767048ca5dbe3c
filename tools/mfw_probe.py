#!/usr/bin/env python3
"""One device-resident multi-frame launch at B streams (for the MFW_STAMPS
diagnostic build: LPCNET_LIB_VARIANT=mfwst prints per-wave work / wait)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
for kv in sys.argv[3:]:
    k, v = kv.split("=", 1)
    os.environ[k] = v
import lpcnet_amd as L  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 3072
F = int(sys.argv[2]) if len(sys.argv) > 2 else 6
blob = L.synthetic_model(1, 0, skewed=os.environ.get("PROBE_SKEWED") == "1")
feats = np.ascontiguousarray(np.stack([L.synthetic_features(s, F)[:, :20] for s in range(B)], 1), np.float32)
b = L.LPCNetBatch(B, 0, blob)
d_f = b.device_alloc(feats.nbytes)
d_p = b.device_alloc(F * B * 160 * 2)
b.h2d(d_f, feats)
b.reset_timers(1)
b.synthesize_frames(None, d_f, d_p, F)
b.sync()
print("kernel", b.info().kernel_name, "ms", b.kernel_ms(0), "frames", b.kernel_frames(0))
