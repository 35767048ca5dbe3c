#!/usr/bin/env python3
"""Aggregate throughput of the drop-in API (include/lpcnet.h) from T
concurrent threads, one LPCNetState each (the shared pool coalesces their
lpcnet_synthesize calls), against LPCNetBatch(T) with host I/O frame by frame
and the device-resident multi-frame path.  Writes gpurun_out/dropin.json."""
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import lpcnet_amd as L  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 64
F = int(sys.argv[2]) if len(sys.argv) > 2 else 100
blob = L.synthetic_model(1, 0)
feats = [L.synthetic_features(t, F)[:, :20] for t in range(T)]
out = {"threads": T, "frames": F}

nets = [L.LPCNet(blob) for _ in range(T)]
for n in nets:
    n.synthesize(feats[0][0])
go = threading.Barrier(T + 1)


def run(t):
    go.wait()
    for f in range(F):
        nets[t].synthesize(feats[t][f])


th = [threading.Thread(target=run, args=(t,)) for t in range(T)]
for x in th:
    x.start()
go.wait()
t0 = time.perf_counter()
for x in th:
    x.join()
dt = time.perf_counter() - t0
import ctypes as C  # noqa: E402
la, rq, ns = C.c_long(0), C.c_long(0), C.c_int(0)
L.lib.lpcnet_mi355x_pool_stats(C.c_void_p(nets[0]._st), C.byref(la), C.byref(rq), C.byref(ns))
out["dropin_threads"] = {"samples_per_s": T * F * 160 / dt, "launches": la.value, "requests": rq.value,
                         "mean_coalesced_streams": rq.value / max(la.value, 1)}

b = L.LPCNetBatch(T, 0, blob)
allf = np.ascontiguousarray(np.stack(feats, 1))
b.synthesize(allf[0])
t0 = time.perf_counter()
for f in range(F):
    b.synthesize(allf[f])
dt = time.perf_counter() - t0
out["batch_host_io"] = {"samples_per_s": T * F * 160 / dt}
df = b.device_alloc(allf.nbytes)
dp = b.device_alloc(F * T * 160 * 2)
b.h2d(df, allf)
b.reset()
t0 = time.perf_counter()
b.synthesize_frames(None, df, dp, F)
b.sync()
dt = time.perf_counter() - t0
out["batch_device_frames"] = {"samples_per_s": T * F * 160 / dt}
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "dropin.json"), "w"), indent=1)
print(json.dumps(out))
