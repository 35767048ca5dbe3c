"""Trained-model sparsity masks on the GPU.  training_tf2/lpcnet.py:140-160
(Sparsify) keeps GRU_A blocks by a GLOBAL per-gate energy threshold, so a
trained model's block rows can be far longer than the mean (the synthetic
`skewed` generator reproduces that: rows of 60-96 blocks).  Such models
must run bit-exactly and without falling off the fast kernels:

* int8: mf_kernel splits rows longer than its own cap into pieces hosted by
  other lane groups, whose int32 partial sums merge exactly (engine.cpp
  mf_plan); LPCNET_MF_FORCE_SPLIT exercises the same machinery on the
  default model against the golden fixture;
* saturating int8 / fp32 with long rows: the lockstep kernel with its
  weight sections in global memory (the image no longer fits LDS), and
  fp_kernel with streamed slots.
PCM, traced logits and final GRU states against the CPU oracle, tolerance 0."""
import os

import numpy as np
import pytest

import lpcnet_amd as L
import oracle_lib as O

pytestmark = pytest.mark.gpu


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


def feats(stream, nframes):
    return L.synthetic_features(stream, nframes)[:, :20]


def _frames(b, allf, f0, f1):
    part = np.ascontiguousarray(allf[f0:f1])
    F, B = part.shape[:2]
    df = b.device_alloc(part.nbytes)
    dp = b.device_alloc(F * B * 160 * 2)
    b.h2d(df, part)
    b.synthesize_frames(part, df, dp, F)
    b.sync()
    got = np.zeros((F, B, 160), np.int16)
    b.d2h(got, dp)
    b.device_free(df)
    b.device_free(dp)
    return got


def test_forced_split_matches_golden(require_gpu, monkeypatch):
    """mf_kernel's split path on the default model (every row split at the
    smallest own cap that leaves pieces) == the golden fixture bit for bit:
    PCM, traced logits, conditioning, final GRU states."""
    monkeypatch.setenv("LPCNET_MF_FORCE_SPLIT", "1")
    G = np.load(os.path.join(O.GOLDEN, "streams_int8.npz"))
    b = L.LPCNetBatch(len(G["streams"]), 0, L.synthetic_model(1, 0))
    assert b.info().quad_path == 4
    b.set_trace(True)
    for fr in range(G["pcm"].shape[1]):
        pcm = b.synthesize(G["features"][:, fr, :20])
        assert np.array_equal(pcm, G["pcm"][:, fr]), fr
        if 2 <= fr < 6:
            lg, ex = b.get_trace(160)
            assert np.array_equal(ex[0], G["trace_exc"][fr - 2])
            assert np.array_equal(bits(lg[0]), bits(G["trace_logits"][fr - 2]))
    st = b.get_state(0)
    assert np.array_equal(bits(st["gru_a_state"]), bits(G["final_gru_a_state"]))
    assert np.array_equal(bits(st["gru_b_state"]), bits(G["final_gru_b_state"]))


def test_forced_long_fp32_matches_golden(require_gpu, monkeypatch):
    """fp_kernel's long form (every z/r/h slot streamed from global memory)
    on the default fp32 model == the golden fixture, PCM and final states."""
    monkeypatch.setenv("LPCNET_FP_FORCE_LONG", "1")
    G = np.load(os.path.join(O.GOLDEN, "streams_fp32.npz"))
    b = L.LPCNetBatch(len(G["streams"]), 0, L.synthetic_model(1, 1))
    info = b.info()
    assert info.quad_path == 5 and info.long_rows == 1
    for fr in range(G["pcm"].shape[1]):
        assert np.array_equal(b.synthesize(G["features"][:, fr, :20]), G["pcm"][:, fr]), fr
    st = b.get_state(0)
    assert np.array_equal(bits(st["gru_a_state"]), bits(G["final_gru_a_state"]))
    assert np.array_equal(bits(st["gru_b_state"]), bits(G["final_gru_b_state"]))


@pytest.mark.parametrize("B", [1, 70])
def test_skewed_fp32_on_fp_kernel(require_gpu, B):
    """Skewed fp32 model: the automatic kernel is fp_kernel's long form,
    against the oracle (host frames, then the overlapped device path)."""
    F = 8
    blob = L.synthetic_model(1, 1, skewed=True)
    b = L.LPCNetBatch(B, 0, blob)
    assert b.info().quad_path == 5 and b.info().long_rows == 1
    allf = np.ascontiguousarray(np.stack([feats(s, F) for s in range(B)], 1))
    out = np.concatenate([np.stack([b.synthesize(allf[f]) for f in range(3)]), _frames(b, allf, 3, F)], 0)
    assert np.abs(out[3:].astype(np.float64)).mean() > 100
    for s in (0, B - 1):
        o = O.Oracle(blob, 1)
        exp = np.stack([o.synthesize(allf[f, s]) for f in range(F)])
        assert np.array_equal(out[:, s], exp), s


@pytest.mark.parametrize("B,check", [(1, (0,)), (70, (0, 69)), (256, (0, 255)), (1030, (0, 517, 1029))])
def test_skewed_int8_on_matrix_cores(require_gpu, B, check):
    """Skewed (Sparsify-like) int8 model: the automatic kernel is mf_kernel
    (split rows), at 1, 2 (70 streams: 1 per workgroup) and 4 streams per
    workgroup; above one mf_kernel<4> round (1030 streams, ragged) the wide
    kernel's split form (round 6); host frames then the multi-frame device
    path, against the oracle."""
    F = 8
    blob = L.synthetic_model(1, 0, skewed=True)
    b = L.LPCNetBatch(B, 0, blob)
    want = 7 if B > 1024 else 4
    assert b.info().quad_path == want and b.info().long_rows == 1, b.info().quad_path
    allf = np.ascontiguousarray(np.stack([feats(s, F) for s in range(B)], 1))
    out = np.concatenate([np.stack([b.synthesize(allf[f]) for f in range(3)]), _frames(b, allf, 3, F)], 0)
    assert np.abs(out[3:].astype(np.float64)).mean() > 100
    for s in check:
        o = O.Oracle(blob, 0)
        exp = np.stack([o.synthesize(allf[f, s]) for f in range(F)])
        assert np.array_equal(out[:, s], exp), s
        a, g = o.state()
        st = b.get_state(s)
        assert np.array_equal(bits(st["gru_a_state"]), bits(a)), s
        assert np.array_equal(bits(st["gru_b_state"]), bits(g)), s


@pytest.mark.parametrize("variant,sat,kernel", [(0, True, 0), (1, False, 0), (1, False, 1), (0, False, 1)])
@pytest.mark.parametrize("B", [3, 300])
def test_skewed_other_kernels(require_gpu, variant, sat, kernel, B):
    """Skewed saturating int8 (lockstep kernel, weights from global memory)
    and skewed fp32 (automatic kernel; lockstep), against the oracle."""
    F = 6
    blob = L.synthetic_model(1, variant, saturating=sat, skewed=True)
    b = L.LPCNetBatch(B, 0, blob)
    b.set_kernel(kernel)
    allf = np.stack([feats(s, F) for s in range(B)], 1)
    out = np.stack([b.synthesize(allf[f]) for f in range(F)], 0)
    assert np.abs(out[3:].astype(np.float64)).mean() > 100
    for s in (0, B - 1):
        exp = O.synth_stream(blob, allf[:, s], variant)
        assert np.array_equal(out[:, s], exp), s


def test_forced_split_mf2_matches_golden(require_gpu, monkeypatch):
    """mf2_kernel's split form (two staggered groups, one hosted-sum buffer
    per group) on the default model, every row split, at the fixture's three
    streams (LPCNET_MF2=1 takes mf2 at any batch): PCM and final GRU states
    == the golden fixture."""
    monkeypatch.setenv("LPCNET_MF_FORCE_SPLIT", "1")
    monkeypatch.setenv("LPCNET_MF2", "1")
    G = np.load(os.path.join(O.GOLDEN, "streams_int8.npz"))
    b = L.LPCNetBatch(len(G["streams"]), 0, L.synthetic_model(1, 0))
    info = b.info()
    assert info.quad_path == 6 and info.long_rows == 1, (info.quad_path, info.long_rows)
    for fr in range(G["pcm"].shape[1]):
        assert np.array_equal(b.synthesize(G["features"][:, fr, :20]), G["pcm"][:, fr]), fr
    for s in range(len(G["streams"])):
        st = b.get_state(s)
        if s == 0:
            assert np.array_equal(bits(st["gru_a_state"]), bits(G["final_gru_a_state"]))
            assert np.array_equal(bits(st["gru_b_state"]), bits(G["final_gru_b_state"]))


@pytest.mark.parametrize("B,check", [(2048, (0, 1031, 2047)), (8192, (0, 4099, 8191))])
def test_skewed_int8_on_mf2(require_gpu, monkeypatch, B, check):
    """Skewed (trained-like) int8 model at mf2_kernel's batch sizes with the
    wide kernel's split form off (LPCNET_NO_MFW_SPLIT=1; the automatic
    choice is covered by test_wide_kernel_split_form_matches_oracle):
    mf2_kernel's split form; host frames then the chunked multi-frame device
    path, PCM and final states against the oracle."""
    monkeypatch.setenv("LPCNET_NO_MFW_SPLIT", "1")
    F = 7
    blob = L.synthetic_model(1, 0, skewed=True)
    b = L.LPCNetBatch(B, 0, blob)
    info = b.info()
    assert info.quad_path == 6 and info.long_rows == 1, info.quad_path
    allf = np.ascontiguousarray(np.stack([feats(s, F) for s in range(B)], 1))
    out = np.concatenate([np.stack([b.synthesize(allf[f]) for f in range(3)]), _frames(b, allf, 3, F)], 0)
    assert np.abs(out[3:].astype(np.float64)).mean() > 100
    for s in check:
        o = O.Oracle(blob, 0)
        exp = np.stack([o.synthesize(allf[f, s]) for f in range(F)])
        assert np.array_equal(out[:, s], exp), s
        a, g = o.state()
        st = b.get_state(s)
        assert np.array_equal(bits(st["gru_a_state"]), bits(a)), s
        assert np.array_equal(bits(st["gru_b_state"]), bits(g)), s
