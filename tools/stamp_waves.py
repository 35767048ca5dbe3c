"""Per-wave mean s_memtime phase stamps of one stamped frame (diagnostic):
python tools/stamp_waves.py B [default|skewed]  -> one row per wave, slots 0..15
(cycles per sample; slot meanings: mf_kernel.hip stamp() calls)."""
import os, sys
import numpy as np
sys.path.insert(0, os.getcwd())
import lpcnet_amd as L

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
blob = L.synthetic_model(1, 0, skewed=len(sys.argv) > 2 and sys.argv[2] == "skewed")
b = L.LPCNetBatch(B, 0, blob)
F = 4
allf = np.stack([L.synthetic_features(s, F)[:, :20] for s in range(B)], 1)
for f in range(F - 1):
    b.synthesize(allf[f])
b.set_stamps(True)
b.synthesize(allf[F - 1])
st = b.get_stamps().astype(np.float64)
print(b.info().kernel_name, os.environ.get("LPCNET_LIB_VARIANT", "default"))
b.close()
n = max(st[:, :, 7].max(), 1)
per = (st / n).mean(axis=0)
print("wave " + " ".join(f"{k:>6d}" for k in range(16)))
for w in range(per.shape[0]):
    print(f"w{w:<3d} " + " ".join(f"{v:6.0f}" for v in per[w]))
