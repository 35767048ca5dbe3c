#!/usr/bin/env python3
"""Per-frame host-I/O loop (lpcnet_batch_synthesize once per frame) at B
streams, for a rocprofv3 kernel trace of the live path: prints the mean wall
time per frame.  Usage: live_probe.py [B] [frames] [host] [env=val ...]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
host = "host" in sys.argv[3:]  # the batch's own pinned buffers (lpcnet_batch_host_features / _pcm)
for kv in sys.argv[3:]:
    if "=" in kv:
        k, v = kv.split("=", 1)
        os.environ[k] = v
import lpcnet_amd as L  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
F = int(sys.argv[2]) if len(sys.argv) > 2 else 30
blob = L.synthetic_model(1, 0)
feats = np.ascontiguousarray(np.stack([L.synthetic_features(s, F)[:, :20] for s in range(B)], 1), np.float32)
b = L.LPCNetBatch(B, 0, blob)
if host:
    hf = b.host_features()

    def tick(f):
        np.copyto(hf, feats[f])
        return b.synthesize_host()
else:
    def tick(f):
        return b.synthesize(feats[f])
for f in range(F):
    tick(f)
b.reset()
per = []
for f in range(F):
    t0 = time.perf_counter()
    tick(f)
    per.append(time.perf_counter() - t0)
per = np.array(per[3:])
print({"B": B, "ms_per_frame": per.mean() * 1e3, "p50": float(np.median(per)) * 1e3,
       "samples_per_s": B * 160 / per.mean(), "kernel": b.info().kernel_name})
