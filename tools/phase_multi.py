#!/usr/bin/env python3
"""Stamped critical path of the matrix-core sample kernel in one
multi-frame launch (lpcnet_batch_synthesize_frames) against single-frame
launches: cycles per sample by phase, and the event-timed ms per frame.
Diagnostic only (stamps are off in every timed run)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import lpcnet_amd as L  # noqa: E402

NAMES = ["X->Y", "waitY", "Y->X", "-", "rest", "waitX"]


def run(B, multi, F=20):
    blob = L.synthetic_model(1, 0)
    b = L.LPCNetBatch(B, 0, blob)
    allf = np.ascontiguousarray(np.stack([L.synthetic_features(s, F + 3)[:, :20] for s in range(B)], 1))
    for f in range(3):
        b.synthesize(allf[f])
    b.set_stamps(True)
    b.reset_timers(1)
    if multi:
        part = np.ascontiguousarray(allf[3:])
        df = b.device_alloc(part.nbytes)
        dp = b.device_alloc(F * B * 160 * 2)
        b.h2d(df, part)
        b.synthesize_frames(part, df, dp, F)
        b.sync()
    else:
        for f in range(3, F + 3):
            b.synthesize(allf[f])
    kms, kn = b.kernel_ms(0)
    kf = b.kernel_frames(0)
    st = b.get_stamps().astype(np.float64)
    n = max(st[:, :, 7].max(), 1)
    per = st / n
    frame_ms = kms / max(kf, 1)
    clock = st[:, :, 6].max() / (kms / max(kn, 1) * 1e-3) / 1e9 if multi else st[:, :, 6].max() / (frame_ms * 1e-3) / 1e9
    print(f"B={B} {'multi ' if multi else 'single'} launches={kn} frames={kf} ms/frame={frame_ms:.4f} "
          f"samples/stamp={n:.0f} clock~{clock:.2f} GHz")
    for w in (0, 4, 6):
        row = per[:, w, :].mean(0)
        print(f"   wave {w}: " + " ".join(f"{NAMES[j]}={row[j]:7.0f}" for j in range(6) if NAMES[j] != "-") +
              f"  loop={row[6]:7.0f}")
    b.close()


if __name__ == "__main__":
    for B in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,1024").split(",")]:
        run(B, False)
        run(B, True)
