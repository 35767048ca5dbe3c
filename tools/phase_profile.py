#!/usr/bin/env python3
"""Per-phase cycle breakdown of the sample kernels (s_memtime stamps).
Diagnostic build path only: the stamps are off in every timed run."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import lpcnet_amd as L  # noqa: E402

NAMES = {1: ["B(gru_a)", "wait1", "C(gru_b)", "wait2", "F(sample)", "wait3"],
         3: ["X->Y", "waitY", "Y->Z", "waitZ", "Z->X", "waitX"],
         4: ["X->Y", "waitY", "Y->X", "-", "rest", "waitX"]}
# fp_kernel stamps (index: name), GRU_A waves / sampler wave
FP_A = {5: "top", 0: "wait_ix", 1: "gathers", 2: "zr_chain", 3: "elem+pub", 4: "wait_all", 8: "h_chain"}
FP_S = {0: "pre", 1: "wait_w0", 2: "gru_b", 3: "elem+bcast", 4: "walk+pub", 8: "post"}


def profile(B, variant=0, kernel=1):
    blob = L.synthetic_model(1, variant)
    b = L.LPCNetBatch(B, 0, blob)
    b.set_kernel(kernel)
    F = 4
    allf = np.stack([L.synthetic_features(s, F)[:, :20] for s in range(B)], 1)
    for f in range(3):
        b.synthesize(allf[f])
    b.set_stamps(True)
    b.reset_timers(True)
    b.synthesize(allf[3])
    kms, kn = b.kernel_ms(0)
    st = b.get_stamps().astype(np.float64)  # [g][8][16]
    n = max(st[:, :, 7].max(), 1)
    per = st / n  # cycles per sample
    info = b.info()
    k = {3: 3, 4: 4, 5: 5}.get(info.quad_path, 1)
    print(f"B={B} variant={variant} kernel={info.kernel_name} groups={st.shape[0]}"
          f"  sample kernel {kms / max(kn, 1) * 1e3:.0f} us -> s_memtime rate "
          f"{st[:, :, 6].max() / max(kms / max(kn, 1), 1e-9) / 1e6:.2f} GHz (stamped run)")
    for w in range(8 if k != 5 else 0):
        row = per[:, w, :].mean(0)
        if row[6] == 0:
            continue
        print(f"  wave {w}: " + " ".join(f"{NAMES[k][j]}={row[j]:7.0f}" for j in range(6)) + f"  loop={row[6]:7.0f}")
    if k == 5:
        sw = int(os.environ.get("FP_SAMPLER_HW", "3"))  # must match the build
        role = ({3: "sampler", 0: "g0", 1: "g1", 2: "g2", 6: "g3", 5: "g4", 4: "g5"} if sw == 3 else
                {0: "sampler", 3: "g0", 1: "g1", 2: "g2", 6: "g3", 5: "g4", 4: "g5"})  # fp_gru_a_wave
        for w in sorted(role, key=lambda x: (role[x] != "sampler", role[x])):
            row = per[:, w, :].mean(0)
            names = FP_S if role[w] == "sampler" else FP_A
            print(f"  {role[w]:>7}: " + " ".join(f"{v}={row[j]:6.0f}" for j, v in names.items()) + f"  loop={row[6]:7.0f}")
    fs = b.get_frame_stamps().astype(np.float64).mean(0)
    print("  frame kernel (cycles): prologue=%.0f conv1=%.0f conv2=%.0f dense1=%.0f dense2=%.0f proj=%.0f epilogue=%.0f total=%.0f" %
          tuple(fs[:8]))
    if k == 4:
        print("  GRU_A X->Y gathers (to last arrival): " + " ".join("w%d=%.0f" % (w, per[:, w, 10].mean()) for w in range(6)))
    if k in (3, 4):
        row = per[:, 6, :].mean(0)
        print("  sampler detail (wave 6): gru_b=%.0f [mfma %.0f sig %.0f tanh+ %.0f] bcast=%.0f walk=%.0f post=%.0f | X->Y finish=%.0f" %
              (row[8] + row[10] + row[14], row[10], row[14], row[8], row[9], row[11], row[12], row[13]))
    if k == 1:
        row = per[:, 0, :].mean(0)
        print("  F detail (wave 0): gru_b=%.0f bcast=%.0f lvl0-3=%.0f lvl4-7=%.0f out=%.0f pre=%.0f" %
              (row[8], row[9], row[10], row[11], row[12], row[4]))
    b.close()


if __name__ == "__main__":
    kerns = [int(k) for k in sys.argv[1].split(",")] if len(sys.argv) > 1 else [3, 4]
    for kern in kerns:
        if kern == 5:
            profile(1, 1, 5)
            continue
        for B in (1, 1024):
            profile(B, 0, kern)
    if len(sys.argv) <= 2 or sys.argv[2] != "nofp32":
        profile(1, 1)
