#!/usr/bin/env python3
"""Tabulates the GPU box host CPU's rcpps (_mm256_rcp_ps, vec_avx.h:408,437)
through the reference's compiled kernels (oracle/_ref, a checker, not the
product) and compares it with the committed Intel table
tests/golden/rcp_x86.bin.  Writes gpurun_out/box_rcp.json and .bin."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as O  # noqa: E402
import bench  # noqa: E402

tab, bad = O.ref_rcp_table()
diff = np.nonzero(tab != O.RCP_TABLE)[0]
out = {"cpu_model": bench.cpu_model(), "violations_of_11bit_property": int(bad), "entries_differing_from_intel": int(len(diff)),
       "first_differences": [[int(i), hex(int(O.RCP_TABLE[i])), hex(int(tab[i]))] for i in diff[:8]]}
# exponent invariance: rcp(x * 2^e) == rcp(x) * 2^-e over a spread of exponents
xs = np.frombuffer((np.arange(2048, dtype=np.uint32) << 12 | 0x3f800000 | 0x7ff).astype(np.uint32).tobytes(), np.float32)
inv = 0
for e in (-60, -20, -3, 3, 20, 60):
    s = np.float32(2.0) ** e
    for x in xs[::37]:
        a, b = O.ref_rcp(float(x * s)), np.float32(O.ref_rcp(float(x))) / s
        inv += int(np.float32(a) != np.float32(b))
out["exponent_invariance_violations"] = inv
# the full mantissa table: on how many top mantissa bits does it depend?
import ctypes as C  # noqa: E402
full = np.zeros(1 << 23, np.uint32)
O._ref.ref_rcp_full.argtypes = [C.c_void_p]
O._ref.ref_rcp_full(full.ctypes.data)
for k in range(11, 24):
    blocks = full.reshape(1 << k, -1)
    if np.all(blocks == blocks[:, :1]):
        out["depends_on_top_mantissa_bits"] = k
        break
out["full_table_distinct_values"] = int(len(np.unique(full)))
rel = full.view(np.float32).astype(np.float64) * (1.0 + np.arange(1 << 23) / 2.0 ** 23) - 1.0
out["max_rel_error"] = float(np.abs(rel).max())
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "box_rcp_full.npz"), full=full)
tab.tofile(os.path.join(ROOT, "gpurun_out", "box_rcp.bin"))
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "box_rcp.json"), "w"), indent=1)
print(json.dumps(out))
