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
