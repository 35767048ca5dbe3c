"""lpc_from_cepstrum (freq.c:310-320) on the GPU (lpcnet_amd/csrc/lpc_kernel.hip).

Bit-exactness rests on two facts:
  * every operation but the band power is an IEEE float/double op restated in
    the reference's order (idct, band interpolation, the 320-point kiss FFT,
    noise floor / lag window, float Levinson-Durbin);
  * the band power (float)(pow(10, E) * compensation) uses pow10_dd.h instead
    of glibc's pow; oracle/checks/pow10_exhaustive.c proves the two give the
    same float for all 2^32 float inputs and every compensation factor
    (full run: profiles/r02/pow10_exhaustive.log; the CPU test below re-runs a
    strided sample, LPCNET_POW10_FULL=1 runs all of it).
The -m gpu tests pin the device kernel against the reference's own compiled
lpc_from_cepstrum (oracle/_ref, or the golden vectors it produced)."""
import os
import subprocess

import numpy as np
import pytest

import lpcnet_amd as L
import oracle_lib as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K = np.load(os.path.join(O.GOLDEN, "kernels.npz"))
COMP = np.array([0.8, 1, 1, 1, 1, 1, 1, 1, 0.666667, 0.5, 0.5, 0.5, 0.333333, 0.25, 0.25, 0.2, 0.166667, 0.173913],
                np.float32)


def test_pow10_dd_matches_glibc_pow(tmp_path):
    exe = tmp_path / "pow10x"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-pthread", "-o", str(exe),
                    os.path.join(ROOT, "oracle", "checks", "pow10_exhaustive.c"), "-lm"], check=True)
    stride = "1" if os.environ.get("LPCNET_POW10_FULL") else "61"
    r = subprocess.run([str(exe), str(min(8, os.cpu_count() or 1)), stride], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:]
    assert " 0 mismatches" in r.stdout
    log = open(os.path.join(ROOT, "profiles", "r02", "pow10_exhaustive.log")).read()
    assert "stride 1), 0 mismatches" in log


def _ref_lpc(ceps):
    k = O.kernel_table(O.ref_kernels() if O.have_ref() else O.port_kernels())
    out = np.zeros((len(ceps), 16), np.float32)
    for i in range(len(ceps)):
        c = np.ascontiguousarray(ceps[i], np.float32)
        k.lpc_from_cepstrum(out[i].ctypes.data, c.ctypes.data)
    return out


def test_port_lpc_matches_golden():
    """the CPU checker the GPU test falls back to (when oracle/_ref is absent) is pinned"""
    ceps = np.ascontiguousarray(K["lpc_ceps"], np.float32)
    k = O.kernel_table(O.port_kernels())
    for i in range(len(ceps)):
        out = np.zeros(16, np.float32)
        k.lpc_from_cepstrum(out.ctypes.data, ceps[i].ctypes.data)
        assert np.array_equal(out.view(np.uint32), K["lpc_out"][i].view(np.uint32)), i


@pytest.mark.gpu
def test_device_lpc_matches_reference_golden(require_gpu):
    ceps = np.ascontiguousarray(K["lpc_ceps"], np.float32)[:, :18]
    got = L.device_lpc(ceps)
    assert np.array_equal(got.view(np.uint32), np.asarray(K["lpc_out"], np.float32).view(np.uint32))


@pytest.mark.gpu
def test_device_lpc_matches_reference_wide(require_gpu):
    """synthetic features of 2,000 streams x 4 frames, plus extreme cepstra
    (huge / tiny band energies, all-zero, single-band spikes)"""
    ceps = [L.synthetic_features(s, 4)[:, :18] for s in range(2000)]
    rng = np.random.default_rng(11)
    ext = np.concatenate([rng.normal(0, 8, (200, 18)), rng.uniform(-60, 60, (200, 18)), np.zeros((1, 18)),
                          np.eye(18) * 40, -np.eye(18) * 40]).astype(np.float32)
    ceps = np.ascontiguousarray(np.concatenate(ceps + [ext]), np.float32)
    got = L.device_lpc(ceps)
    exp = _ref_lpc(ceps)
    # Band energies beyond float range give inf - inf in the FFT: x86 then
    # produces its "indefinite" NaN (0xFFC00000), the GPU the canonical
    # 0x7FC00000.  Where the reference is NaN the device must be NaN; every
    # other value must match bit for bit.
    nan = np.isnan(exp)
    assert np.array_equal(np.isnan(got), nan)
    bad = np.flatnonzero(np.any((got.view(np.uint32) != exp.view(np.uint32)) & ~nan, axis=1))
    assert bad.size == 0, f"{bad.size} rows differ, first {bad[:5]}"
    assert nan.any(axis=1).sum() < 250  # the uniform(-60, 60) rows only


@pytest.mark.gpu
def test_device_band_power_matches_glibc(require_gpu):
    """(float)(pow(10, E) * comp) on the device (op 9) against numpy's (glibc) pow,
    over a dense sweep of the finite range and random bit patterns"""
    rng = np.random.default_rng(5)
    sweep = np.linspace(-50, 45, 3_000_000, dtype=np.float32)
    bitsr = rng.integers(0, 2 ** 32, 1_000_000, dtype=np.uint64).astype(np.uint32).view(np.float32)
    x = np.ascontiguousarray(np.concatenate([sweep, bitsr, np.array([np.inf, -np.inf, 0, -0.0, 38.53184], np.float32)]))
    x = x[: len(x) // 18 * 18]
    got = L.device_numerics(9, x)
    comp = np.tile(COMP, len(x) // 18).astype(np.float64)
    with np.errstate(over="ignore", invalid="ignore"):
        exp = (np.power(10.0, x.astype(np.float64)) * comp).astype(np.float32)
    nan = np.isnan(exp)
    assert np.array_equal(got[~nan], exp[~nan].view(np.uint32))
    assert np.all(np.isnan(got[nan].view(np.float32)))
