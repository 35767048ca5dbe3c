#!/usr/bin/env python3
"""Generates the golden fixtures in tests/golden/ (run in the build container).

Every expected value here is produced by the reference's OWN compiled
arithmetic kernels -- /root/reference/src vec_avx.h (AVX2 DOT_PROD and
DISABLE_DOT_PROD builds), common.h, kiss99.c, freq.c + kiss_fft.c +
lpcnet_tables.c -- built in place by oracle/Makefile into
oracle/_ref/libref_kernels.so.  End-to-end PCM composes those kernels with the
oracle's restatement of lpcnet.c / nnet.c (which cannot be compiled from the
reference: they need the generated nnet_data.h that the reference does not
ship).  Inputs are the product's deterministic synthetic model and features,
whose SHA-256 is recorded so that drift of the generator is detected.

Usage: python3 tests/golden/make_golden.py
"""
import ctypes as C
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import oracle_lib as O  # noqa: E402
import lpcnet_amd as L  # noqa: E402

assert O.have_ref(), "oracle/_ref/libref_kernels.so missing: run `make -C oracle` with /root/reference present"
REF = O.kernel_table(O.ref_kernels())
rng = np.random.default_rng(20251015)


def fptr(a):
    return a.ctypes.data


def kernels_fixture():
    d = {}
    tab, bad = O.ref_rcp_table()
    assert bad == 0
    assert np.array_equal(tab, O.RCP_TABLE), "rcp table of this CPU differs from tests/golden/rcp_x86.bin"
    # activations: dense grid, random, and special values
    x = np.concatenate([np.linspace(-12, 12, 24001, dtype=np.float32),
                        rng.normal(0, 4, 20000).astype(np.float32),
                        np.array([0.0, -0.0, 1e-30, -1e-30, 1e-8, 60.0, -60.0, 1e4, -1e4, 1e10, -1e10,
                                  3.4e38, -3.4e38, np.inf, -np.inf, np.nan], np.float32)])
    x = np.ascontiguousarray(x[: len(x) // 8 * 8])
    th = np.zeros_like(x)
    sg = np.zeros_like(x)
    REF.vec_tanh(fptr(th), fptr(x), len(x))
    REF.vec_sigmoid(fptr(sg), fptr(x), len(x))
    d["act_x"], d["act_tanh"], d["act_sigmoid"] = x, th, sg
    # quantization
    q = np.concatenate([np.linspace(-1.2, 1.2, 4001, dtype=np.float32), rng.uniform(-1, 1, 4000).astype(np.float32)])
    q = np.ascontiguousarray(q[: len(q) // 8 * 8])
    d["quant_x"], d["quant_u8"] = q, O.quantize_u8(q, ref=True)
    # block-sparse int8 (normal and saturating weights)
    for tag, sat in (("", False), ("_sat", True)):
        rows, cols = 96, 64
        idx = []
        for rb in range(rows // 8):
            pos = sorted(rng.choice(cols // 4, size=int(rng.integers(0, cols // 4 + 1)), replace=False) * 4)
            idx += [len(pos)] + list(pos)
        idx = np.array(idx, np.int32)
        nblk = 0
        p = 0
        while p < len(idx):
            nblk += idx[p]
            p += idx[p] + 1
        lim = 128 if sat else 64
        w = rng.integers(-lim, lim, size=32 * nblk).astype(np.int8)
        if sat:
            w[::7] = 127
            w[1::7] = 127
            w[3::11] = -128
            w[4::11] = -128
        xv = rng.uniform(-1, 1, cols).astype(np.float32)
        if sat:
            xv[::3] = 1.0
        out0 = rng.uniform(-0.5, 0.5, rows).astype(np.float32)
        out = out0.copy()
        REF.sparse8x4_i8(fptr(out), fptr(w), rows, cols, fptr(idx), fptr(xv))
        d["sp8_idx" + tag], d["sp8_w" + tag], d["sp8_x" + tag], d["sp8_in" + tag], d["sp8_out" + tag] = idx, w, xv, out0, out
    # dense int8 (GRU_B recurrent shape 48 x 16)
    w = rng.integers(-64, 64, size=48 * 16).astype(np.int8)
    xv = rng.uniform(-1, 1, 16).astype(np.float32)
    out0 = rng.uniform(-0.5, 0.5, 48).astype(np.float32)
    out = out0.copy()
    REF.dense8x4_i8(fptr(out), fptr(w), 48, 16, fptr(xv))
    d["dn8_w"], d["dn8_x"], d["dn8_in"], d["dn8_out"] = w, xv, out0, out
    # block-sparse fp32
    idx = d["sp8_idx"]
    nblk = len(d["sp8_w"]) // 32
    wf = rng.uniform(-0.5, 0.5, 32 * nblk).astype(np.float32)
    xv = rng.uniform(-1, 1, 64).astype(np.float32)
    out0 = rng.uniform(-0.5, 0.5, 96).astype(np.float32)
    out = out0.copy()
    REF.sparse8x4_f32(fptr(out), fptr(wf), 96, fptr(idx), fptr(xv))
    d["spf_w"], d["spf_x"], d["spf_in"], d["spf_out"] = wf, xv, out0, out
    # sgemv_accum16 (conv1 shape)
    w = rng.uniform(-0.1, 0.1, 252 * 128).astype(np.float32)
    xv = rng.uniform(-1, 1, 252).astype(np.float32)
    out0 = rng.uniform(-0.1, 0.1, 128).astype(np.float32)
    out = out0.copy()
    REF.sgemv16(fptr(out), fptr(w), 128, 252, 128, fptr(xv))
    d["sg16_w"], d["sg16_x"], d["sg16_in"], d["sg16_out"] = w, xv, out0, out
    # u-law
    lx = np.concatenate([np.linspace(-40000, 40000, 16001, dtype=np.float32), rng.normal(0, 3000, 8000).astype(np.float32)])
    d["l2u_x"] = lx
    d["l2u"] = np.array([REF.lin2ulaw(float(v)) for v in lx], np.int32)
    d["u2l"] = np.array([REF.ulaw2lin(float(v)) for v in range(256)], np.float32)
    # kiss99 seeded like lpcnet_reset (lpcnet.c:176-181)
    ctx = (C.c_uint32 * 4)()
    seed = b"LPCNet"
    REF.rng_srand(C.addressof(ctx), seed, len(seed))
    d["kiss99_lpcnet"] = np.array([REF.rng_rand(C.addressof(ctx)) for _ in range(256)], np.uint32)
    # lpc_from_cepstrum
    ceps = np.concatenate([L.synthetic_features(s, 16)[:, :18] for s in range(4)] +
                          [rng.normal(0, 1, (64, 18)).astype(np.float32) * np.array([2.0] + [0.6 / k for k in range(1, 18)], np.float32)])
    ceps = np.ascontiguousarray(ceps, np.float32)
    lpc = np.zeros((len(ceps), 16), np.float32)
    for k in range(len(ceps)):
        REF.lpc_from_cepstrum(fptr(lpc[k]), fptr(ceps[k]))
    d["lpc_ceps"], d["lpc_out"] = ceps, lpc
    np.savez_compressed(os.path.join(HERE, "kernels.npz"), **d)
    print("kernels.npz:", {k: v.shape for k, v in d.items()})


STREAMS = (0, 1, 7)
NFRAMES = 40


def stream_fixture(name, variant, saturating, constants=None, STREAMS=STREAMS, NFRAMES=NFRAMES):
    """constants: (LPC_GAMMA, FEATURES_DELAY, END2END) of a trained model's
    nnet_data.h (dump_lpcnet.py:423-446); None = the dump defaults."""
    blob = L.synthetic_model(1, variant, saturating)
    # the fixture's blob is one the reference's own parser and binders accept
    # (parse_lpcnet_weights.c compiled unmodified, oracle/ref_parse.c)
    assert O.have_ref_parser(), "oracle/_ref/ref_parse_* missing: run `make -C oracle`"
    assert O.ref_parse(blob, variant)[0] == "accept", f"{name}: reference parser rejects the blob"
    d = {"blob_sha256": np.frombuffer(hashlib.sha256(blob).digest(), np.uint8), "variant": np.int32(variant),
         "streams": np.array(STREAMS, np.int32)}
    if constants is not None:
        d["constants"] = np.array(constants, np.float64)
    pcm = np.zeros((len(STREAMS), NFRAMES, 160), np.int16)
    feats = np.zeros((len(STREAMS), NFRAMES, 36), np.float32)
    for si, s in enumerate(STREAMS):
        f = L.synthetic_features(s, NFRAMES)
        feats[si] = f
        o = O.Oracle(blob, variant, O.ref_kernels(), constants)
        logits = np.zeros((4, 160, 8), np.float32)
        exc = np.zeros((4, 160), np.int32)
        rngw = np.zeros((4, 160, 2), np.uint32)
        conds = np.zeros((6, 1152 + 48 + 16), np.float32)
        for fr in range(NFRAMES):
            if si == 0 and 2 <= fr < 6:
                pcm[si, fr], logits[fr - 2], exc[fr - 2], rngw[fr - 2] = o.synthesize(f[fr], trace=True)
            else:
                pcm[si, fr] = o.synthesize(f[fr])
            if si == 0 and fr < 6:
                a, b, lpc = o.frame()
                conds[fr] = np.concatenate([a, b, lpc])
        if si == 0:
            d["trace_logits"], d["trace_exc"], d["trace_rng"], d["frame_cond"] = logits, exc, rngw, conds
            sa, sb = o.state()
            d["final_gru_a_state"], d["final_gru_b_state"] = sa, sb
    d["pcm"], d["features"] = pcm, feats
    # self-check: the portable kernels reproduce the reference kernels end to end
    for si, s in enumerate(STREAMS):
        port = O.synth_stream(blob, feats[si], variant, constants=constants)
        assert np.array_equal(port, pcm[si]), f"{name}: port kernels diverge from reference kernels (stream {s})"
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
    print(name, "rms", float(np.sqrt(np.mean(pcm.astype(np.float64) ** 2))))


# trained-model constants other than the dump defaults (round 3): the
# reference's compiled lpc_weighting (freq.c:299-308) and lpc_from_cepstrum
# drive the LPC ring of each depth; rc2lpc (lpcnet.c:56-80, END2END) is the
# oracle's restatement (lpcnet.c is not compilable here)
CONST_FIXTURES = [("streams_int8_g092_d3", 0, (0.92, 3, 0)), ("streams_int8_g095_d0", 0, (0.95, 0, 0)),
                  ("streams_int8_e2e_g09_d1", 0, (0.9, 1, 1)), ("streams_fp32_g092_d4", 1, (0.92, 4, 0))]

if __name__ == "__main__":
    if sys.argv[1:] == ["constants"]:
        for name, variant, c in CONST_FIXTURES:
            stream_fixture(name, variant, False, c, STREAMS=(0, 5), NFRAMES=12)
        sys.exit(0)
    kernels_fixture()
    stream_fixture("streams_int8", 0, False)
    stream_fixture("streams_fp32", 1, False)
    stream_fixture("streams_int8_sat", 0, True)
    for name, variant, c in CONST_FIXTURES:
        stream_fixture(name, variant, False, c, STREAMS=(0, 5), NFRAMES=12)
