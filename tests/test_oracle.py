"""The CPU checker itself: the oracle's portable kernels against the golden
vectors produced by the reference's own compiled kernels (tests/golden/), and
-- in the build container, where oracle/_ref exists -- directly against them."""
import os

import numpy as np
import pytest

import oracle_lib as O

GOLD = os.path.join(O.GOLDEN, "kernels.npz")
K = np.load(GOLD)
PORT = O.kernel_table(O.port_kernels())


def f32(a):
    return np.ascontiguousarray(a, np.float32)


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


def test_rcp_table_shape_and_monotone():
    t = O.RCP_TABLE.view(np.float32)
    assert np.all((t > 0.5) & (t <= 1.0))
    assert np.all(np.diff(t) <= 0)


def test_activations_bit_exact():
    x = f32(K["act_x"])
    th = np.zeros_like(x)
    sg = np.zeros_like(x)
    PORT.vec_tanh(th.ctypes.data, x.ctypes.data, len(x))
    PORT.vec_sigmoid(sg.ctypes.data, x.ctypes.data, len(x))
    assert np.array_equal(bits(th), bits(K["act_tanh"]))  # NaN payloads too
    assert np.array_equal(bits(sg), bits(K["act_sigmoid"]))


def test_quantize_u8():
    assert np.array_equal(O.quantize_u8(K["quant_x"]), K["quant_u8"])


@pytest.mark.parametrize("tag", ["", "_sat"])
def test_sparse_int8(tag):
    out = f32(K["sp8_in" + tag]).copy()
    w = np.ascontiguousarray(K["sp8_w" + tag])
    idx = np.ascontiguousarray(K["sp8_idx" + tag])
    x = f32(K["sp8_x" + tag])
    PORT.sparse8x4_i8(out.ctypes.data, w.ctypes.data, 96, 64, idx.ctypes.data, x.ctypes.data)
    assert np.array_equal(bits(out), bits(K["sp8_out" + tag]))


def test_dense_int8():
    out = f32(K["dn8_in"]).copy()
    w = np.ascontiguousarray(K["dn8_w"])
    x = f32(K["dn8_x"])
    PORT.dense8x4_i8(out.ctypes.data, w.ctypes.data, 48, 16, x.ctypes.data)
    assert np.array_equal(bits(out), bits(K["dn8_out"]))


def test_sparse_fp32():
    out = f32(K["spf_in"]).copy()
    w = f32(K["spf_w"])
    idx = np.ascontiguousarray(K["sp8_idx"])
    x = f32(K["spf_x"])
    PORT.sparse8x4_f32(out.ctypes.data, w.ctypes.data, 96, idx.ctypes.data, x.ctypes.data)
    assert np.array_equal(bits(out), bits(K["spf_out"]))


def test_sgemv16():
    out = f32(K["sg16_in"]).copy()
    w = f32(K["sg16_w"])
    x = f32(K["sg16_x"])
    PORT.sgemv16(out.ctypes.data, w.ctypes.data, 128, 252, 128, x.ctypes.data)
    assert np.array_equal(bits(out), bits(K["sg16_out"]))


def test_ulaw():
    got = np.array([PORT.lin2ulaw(float(v)) for v in K["l2u_x"]], np.int32)
    assert np.array_equal(got, K["l2u"])
    u2l = np.array([PORT.ulaw2lin(float(v)) for v in range(256)], np.float32)
    assert np.array_equal(bits(u2l), bits(K["u2l"]))


def test_kiss99():
    import ctypes as C
    ctx = (C.c_uint32 * 4)()
    PORT.rng_srand(C.addressof(ctx), b"LPCNet", 6)
    got = np.array([PORT.rng_rand(C.addressof(ctx)) for _ in range(256)], np.uint32)
    assert np.array_equal(got, K["kiss99_lpcnet"])


def test_lpc_from_cepstrum():
    ceps = f32(K["lpc_ceps"])
    for k in range(len(ceps)):
        out = np.zeros(16, np.float32)
        PORT.lpc_from_cepstrum(out.ctypes.data, ceps[k].ctypes.data)
        assert np.array_equal(bits(out), bits(K["lpc_out"][k])), k


@pytest.mark.parametrize("name,variant", [("streams_int8", 0), ("streams_fp32", 1), ("streams_int8_sat", 0)])
def test_oracle_stream_golden(name, variant):
    """End-to-end PCM of the portable oracle == reference-kernel golden PCM
    (first 12 frames of the first fixture stream; full streams in the GPU tests)."""
    import hashlib
    import lpcnet_amd as L
    G = np.load(os.path.join(O.GOLDEN, name + ".npz"))
    blob = L.synthetic_model(1, variant, name.endswith("_sat"))
    assert hashlib.sha256(blob).digest() == G["blob_sha256"].tobytes(), "synthetic model generator drifted"
    o = O.Oracle(blob, variant)
    for fr in range(12):
        if 2 <= fr < 6:
            pcm, lg, ex, rw = o.synthesize(G["features"][0, fr], trace=True)
            assert np.array_equal(bits(lg), bits(G["trace_logits"][fr - 2]))
            assert np.array_equal(ex, G["trace_exc"][fr - 2])
            assert np.array_equal(rw, G["trace_rng"][fr - 2])
        else:
            pcm = o.synthesize(G["features"][0, fr])
        assert np.array_equal(pcm, G["pcm"][0, fr]), fr
        if fr < 6:
            a, b, lpc = o.frame()
            assert np.array_equal(bits(np.concatenate([a, b, lpc])), bits(G["frame_cond"][fr]))


@pytest.mark.parametrize("name,variant", [("streams_int8", 0), ("streams_fp32", 1), ("streams_int8_sat", 0)])
def test_baseline_build_bit_identical(name, variant):
    """The CPU baseline's build of the restatement (-O3 -mavx2 -mfma
    -ffp-contract=off, oracle/Makefile BASE_CFLAGS) with the reference's
    compiled kernels reproduces the golden PCM: the flags change speed only."""
    import lpcnet_amd as L
    if not O.have_avx2_build():
        pytest.skip("liblpcnet_oracle_avx2.so not built")
    G = np.load(os.path.join(O.GOLDEN, name + ".npz"))
    blob = L.synthetic_model(1, variant, name.endswith("_sat"))
    for kernels in ([None, O.ref_kernels()] if O.have_ref() else [None]):
        o = O.Oracle(blob, variant, kernels, avx2_build=True)
        for fr in range(10):
            assert np.array_equal(o.synthesize(G["features"][1, fr]), G["pcm"][1, fr]), fr


CONST_FIXTURES = ["streams_int8_g092_d3", "streams_int8_g095_d0", "streams_int8_e2e_g09_d1", "streams_fp32_g092_d4"]


@pytest.mark.parametrize("name", CONST_FIXTURES)
def test_oracle_model_constants_golden(name):
    """Trained-model constants (LPC_GAMMA, FEATURES_DELAY, END2END;
    dump_lpcnet.py:423-446): the portable oracle reproduces the fixtures made
    with the reference's compiled lpc_weighting / lpc_from_cepstrum, both
    fixture streams, every frame, and the silent first FEATURES_DELAY frames."""
    import lpcnet_amd as L
    G = np.load(os.path.join(O.GOLDEN, name + ".npz"))
    g, d, e = G["constants"]
    variant = int(G["variant"])
    blob = L.synthetic_model(1, variant)
    for si in range(len(G["streams"])):
        o = O.Oracle(blob, variant, constants=(float(g), int(d), int(e)))
        for fr in range(G["pcm"].shape[1]):
            pcm = o.synthesize(G["features"][si, fr])
            assert np.array_equal(pcm, G["pcm"][si, fr]), (si, fr)
            if si == 0 and fr < 6:
                a, b, lpc = o.frame()
                assert np.array_equal(bits(np.concatenate([a, b, lpc])), bits(G["frame_cond"][fr])), fr
        assert np.all(G["pcm"][si, :int(d)] == 0) and np.any(G["pcm"][si, int(d)] != 0)


def test_oracle_rejects_bad_constants():
    import lpcnet_amd as L
    blob = L.synthetic_model(1, 0)
    for c in ((1.0, 5, 0), (1.0, -1, 0), (1.0, 2, 2)):
        with pytest.raises(ValueError):
            O.Oracle(blob, 0, constants=c)


def test_engine_reads_and_validates_constant_records():
    """The engine takes the constants from optional blob records named like
    nnet_data.h's #defines (validated host-side, no GPU), rejects malformed
    or unsupported ones; the records do not disturb any other array."""
    import lpcnet_amd as L
    blob = L.synthetic_model(1, 0)
    L.validate_model(L.with_model_constants(blob, 0.92, 3, True))
    L.validate_model(L.with_model_constants(blob, 1.0, 0, False))
    for kw in ({"features_delay": 5}, {"features_delay": -1}, {"lpc_gamma": float("inf")}):
        with pytest.raises(L.LPCNetError):
            L.validate_model(L.with_model_constants(blob, **kw))
    bad = bytearray(L.with_model_constants(blob, end2end=True))
    bad[-64 + 0] = 7  # END2END = 7
    with pytest.raises(L.LPCNetError, match="END2END"):
        L.validate_model(bytes(bad))


def test_oracle_rejects_bad_blob():
    import lpcnet_amd as L
    blob = bytearray(L.synthetic_model(1, 0))
    with pytest.raises(ValueError):
        O.Oracle(bytes(blob[:-64]), 0)  # truncated record


@pytest.mark.skipif(not O.have_ref(), reason="oracle/_ref not built (reference tree absent)")
def test_port_matches_reference_kernels_live():
    """Build container only: this CPU's rcpps table == the committed one, and the
    portable activations match the reference's compiled vec_avx.h on fresh inputs."""
    tab, bad = O.ref_rcp_table()
    if not np.array_equal(tab, O.RCP_TABLE):
        pytest.skip("host rcpps differs from the pinned x86 table (not the reference host)")
    assert bad == 0
    REF = O.kernel_table(O.ref_kernels())
    rng = np.random.default_rng(7)
    x = f32(rng.normal(0, 6, 8192))
    a, b = np.zeros_like(x), np.zeros_like(x)
    REF.vec_tanh(a.ctypes.data, x.ctypes.data, len(x))
    PORT.vec_tanh(b.ctypes.data, x.ctypes.data, len(x))
    assert np.array_equal(bits(a), bits(b))
