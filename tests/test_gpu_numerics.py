"""The device numerics the sample kernels share (lpcnet_amd/csrc/device_math.h),
evaluated on the GPU through lpcnet_mi355x_device_numerics and pinned
against the reference's own compiled AVX2 kernels (tests/golden/kernels.npz,
made by tests/golden/make_golden.py from /root/reference/src): 44,016
activation inputs including NaN, +-inf, denormals and the saturation
regions, 8,000 quantiser inputs, 24,001 u-law inputs, the first 256 kiss99
draws of lpcnet_reset's seed.  Tolerance: 0 ulp, NaN payloads included."""
import ctypes as C
import os

import numpy as np
import pytest

import lpcnet_amd as L
import oracle_lib as O

pytestmark = pytest.mark.gpu
K = np.load(os.path.join(O.GOLDEN, "kernels.npz"))


def f32bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("op,key", [(0, "act_tanh"), (1, "act_sigmoid"), (2, "act_tanh"), (3, "act_sigmoid")])
def test_activations_bit_exact_on_device(require_gpu, op, key):
    got = L.device_numerics(op, np.ascontiguousarray(K["act_x"], np.float32))
    exp = f32bits(K[key])
    bad = np.flatnonzero(got != exp)
    assert bad.size == 0, f"{bad.size} mismatches, first x={K['act_x'][bad[:4]]}"


def test_quantize_on_device(require_gpu):
    got = L.device_numerics(4, np.ascontiguousarray(K["quant_x"], np.float32))
    assert np.array_equal(got.astype(np.uint8), K["quant_u8"])


def test_lin2ulaw_on_device(require_gpu):
    got = L.device_numerics(5, np.ascontiguousarray(K["l2u_x"], np.float32)).view(np.int32)
    assert np.array_equal(got, K["l2u"])


def test_round_half_up_on_device(require_gpu):
    """lpcnet.c:266 (int)floor(.5 + o) in double, over the clamped output
    range: every integer, every half and random values."""
    rng = np.random.default_rng(7)
    x = np.concatenate([np.arange(-32767, 32768, dtype=np.float32),
                        np.arange(-32767, 32767, dtype=np.float32) + np.float32(0.5),
                        rng.uniform(-32767, 32767, 200000).astype(np.float32),
                        np.nextafter(np.float32(0.5), np.float32(0)) * np.array([1, -1], np.float32)])
    got = L.device_numerics(6, x).view(np.int32)
    exp = np.floor(0.5 + x.astype(np.float64)).astype(np.int32)
    assert np.array_equal(got, exp)


def test_cvtps_epi32_on_device(require_gpu):
    """_mm256_cvtps_epi32: round to nearest even, INT_MIN for NaN and out of range."""
    rng = np.random.default_rng(9)
    special = np.array([0.5, 1.5, 2.5, -0.5, -1.5, -2.5, 2147483520.0, 2147483648.0, -2147483648.0,
                        -2147483904.0, np.inf, -np.inf, np.nan, 1e-45, -0.0], np.float32)
    x = np.concatenate([special, rng.normal(0, 1e4, 100000).astype(np.float32),
                        rng.uniform(-3e9, 3e9, 100000).astype(np.float32)])
    got = L.device_numerics(7, x).view(np.int32)
    r = np.rint(x.astype(np.float64))
    ok = np.isfinite(r) & (r >= -2.0 ** 31) & (r < 2.0 ** 31)
    exp = np.where(ok, np.where(ok, r, 0).astype(np.int64), -2 ** 31).astype(np.int32)
    assert np.array_equal(got, exp)


def test_kiss99_on_device(require_gpu):
    PORT = O.kernel_table(O.port_kernels())
    ctx = (C.c_uint32 * 4)()
    PORT.rng_srand(C.addressof(ctx), b"LPCNet", 6)
    seed = np.array(list(ctx), np.uint32)
    got = L.device_numerics(8, seed, n=256)
    assert np.array_equal(got, K["kiss99_lpcnet"])


def _rcp_x86_expected(bits):
    """rcpps of a Pade denominator from the tabulated x86 instruction
    (tests/golden/rcp_x86.bin: top 11 mantissa bits, exponent-invariant;
    results below 2^-126, +inf and NaN -> +0)."""
    tab = np.fromfile(os.path.join(O.GOLDEN, "rcp_x86.bin"), np.uint32).astype(np.int64)
    t = tab[(bits >> 12) & 0x7FF] + (127 << 23)
    q = t - (bits & 0x7F800000).astype(np.int64)
    return np.where(q < 0x00800000, 0, q).astype(np.uint32)


def test_rcpps_every_prefix_and_exponent_on_device(require_gpu):
    """The device rcpps (device_math.h rcp12_hw: hardware reciprocal of the
    interval midpoint rounded to 12 bits) equals the x86 table for every
    11-bit mantissa prefix at every exponent a Pade denominator can have
    ([952.72, 2^128)), three low-bit patterns each, plus +inf and NaNs."""
    e = np.arange(136, 255, dtype=np.uint32)
    i = np.arange(2048, dtype=np.uint32)
    lo = np.array([0, 0x5A5, 0xFFF], np.uint32)
    bits = ((e[:, None, None] << 23) | (i[None, :, None] << 12) | lo[None, None, :]).ravel()
    bits = bits[bits >= np.float32(952.72399902).view(np.uint32)]
    bits = np.concatenate([bits, np.array([0x7F800000, 0x7FC00000, 0xFFC00000, 0x7F800001], np.uint32)])
    got = L.device_numerics(10, bits)
    exp = _rcp_x86_expected(bits)
    bad = np.flatnonzero(got != exp)
    assert bad.size == 0, f"{bad.size} mismatches, first den bits {bits[bad[:4]]}"


def test_sigmoid_fin_on_device(require_gpu):
    """sigmoid_x86_fin_n (the int8 gates' sigmoid, inputs (float)int32 *
    2^-14 plus such a term: |x| < 2^18) against the reference's compiled
    sigmoid8_approx on the golden inputs of that range and a dense sweep."""
    x = np.ascontiguousarray(K["act_x"], np.float32)
    keep = np.isfinite(x) & (np.abs(x) < 2.0 ** 18)
    got = L.device_numerics(11, x[keep])
    assert np.array_equal(got, f32bits(K["act_sigmoid"])[keep])
    sweep = (np.arange(-2 ** 22, 2 ** 22, 97, dtype=np.int64) * 2.0 ** -14).astype(np.float32)
    assert np.array_equal(L.device_numerics(11, sweep), L.device_numerics(1, sweep))
    assert np.array_equal(L.device_numerics(12, x[keep]), f32bits(K["act_sigmoid"])[keep])
    assert np.array_equal(L.device_numerics(12, sweep), L.device_numerics(1, sweep))
