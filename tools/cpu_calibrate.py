"""CPU-baseline calibration: single-thread speed of
the CPU paths bench.py can time, in THIS container (the survey's Intel Xeon,
where the compiled reference itself was timed at 290 K samples/s/core with
-O3 -march=native -ffp-contract=off):

  port        portable oracle glue (-O2) + portable kernels
  ref         portable oracle glue (-O2) + the reference's own kernels
  ref_avx2    the glue built with the reference's flags (-O3 -mavx2 -mfma)
              + the reference's own kernels   <- bench.py cpu_baseline

Each leg: one pinned thread, one stream, `--seconds` of synthesis.  Prints
one JSON object.  Also checks that the three legs give identical PCM."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import lpcnet_amd as L  # noqa: E402
import oracle_lib as O  # noqa: E402


def leg(blob, variant, kernels, avx2, seconds, feats):
    o = O.Oracle(blob, variant, kernels, avx2_build=avx2)
    o.synthesize(feats[0])
    k, t0 = 1, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        o.synthesize(feats[k % len(feats)])
        k += 1
    dt = time.perf_counter() - t0
    return (k - 1) * 160 / dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--cpu", type=int, default=2)
    a = ap.parse_args()
    os.sched_setaffinity(0, {a.cpu})
    feats = L.synthetic_features(1000, 64)
    out = {"cpu_model": open("/proc/cpuinfo").read().split("model name")[1].split(":")[1].split("\n")[0].strip(),
           "survey_reference_per_core": {"int8 -O3 -march=native -ffp-contract=off": 290e3,
                                         "int8 -O2 -mavx2 -mfma -ffp-contract=off": 214e3}}
    # the container's cores are shared: legs alternate over `rounds` rounds
    # and each keeps its best round (contention only ever slows a leg down)
    for variant, name in ((0, "int8"), (1, "fp32")):
        blob = L.synthetic_model(1, variant)
        pcm = {}
        legs = (("port", None, False), ("ref", O.ref_kernels(), False), ("ref_avx2", O.ref_kernels(), True))
        for lg, k, avx2 in legs:
            o = O.Oracle(blob, variant, k, avx2_build=avx2)
            pcm[lg] = np.stack([o.synthesize(feats[f]) for f in range(12)])
        best = {lg: 0.0 for lg, _, _ in legs}
        for _ in range(a.rounds):
            for lg, k, avx2 in legs:
                best[lg] = max(best[lg], leg(blob, variant, k, avx2, a.seconds / (10 if lg == "port" else 1), feats))
        for lg in best:
            out[f"{name}_{lg}"] = best[lg]
        out[f"{name}_pcm_identical"] = bool(all(np.array_equal(pcm["port"], v) for v in pcm.values()))
    out["ratio_ref_avx2_to_reference_int8_O3_native"] = out["int8_ref_avx2"] / 290e3
    out["ratio_ref_avx2_to_reference_int8_O2_avx2"] = out["int8_ref_avx2"] / 214e3
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
