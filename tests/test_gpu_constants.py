"""Trained-model constants on the GPU: LPC_GAMMA (lpc_weighting,
lpcnet.c:116-118), FEATURES_DELAY (lookahead: LPC ring depth, conv2 clear,
silent first frames; lpcnet.c:101,109-114,239) and END2END (rc2lpc of the
frame network's outputs, lpcnet.c:56-80,107-108) -- the #defines
dump_lpcnet.py:423-446 writes into nnet_data.h from train_lpcnet.py's
--lpc-gamma / --lookahead / --end2end.  The engine reads them from blob
records (or the LPCNET_* environment, or lpcnet_batch_set_model_constants);
every path (per-frame kernels, overlapped frames, chunked frame network with
multi-frame sample launches; mf_kernel, fp_kernel, lockstep kernel) must give
the fixtures' PCM and conditioning bit for bit.  Tolerance 0: integer PCM
identical, floats bit-equal."""
import os

import numpy as np
import pytest

import lpcnet_amd as L
import oracle_lib as O

pytestmark = pytest.mark.gpu
FIXTURES = ["streams_int8_g092_d3", "streams_int8_g095_d0", "streams_int8_e2e_g09_d1", "streams_fp32_g092_d4"]


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


def fixture(name):
    G = np.load(os.path.join(O.GOLDEN, name + ".npz"))
    g, d, e = G["constants"]
    return G, (float(g), int(d), int(e)), int(G["variant"])


def blob_with(variant, c):
    return L.with_model_constants(L.synthetic_model(1, variant), c[0], c[1], bool(c[2]))


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


@pytest.mark.parametrize("name", FIXTURES)
@pytest.mark.parametrize("kernel", [0, 1])
def test_constants_per_frame_match_golden(require_gpu, name, kernel):
    """Blob records -> engine; lpcnet_batch_synthesize frame by frame, the
    automatic kernel (mf_kernel / fp_kernel) and the lockstep kernel."""
    G, c, variant = fixture(name)
    b = L.LPCNetBatch(len(G["streams"]), 0, blob_with(variant, c))
    info = b.info()
    assert (round(info.lpc_gamma, 6), info.features_delay, info.end2end) == (round(c[0], 6), c[1], c[2])
    b.set_kernel(kernel)
    for fr in range(G["pcm"].shape[1]):
        pcm = b.synthesize(G["features"][:, fr, :20])
        assert np.array_equal(pcm, G["pcm"][:, fr]), fr
        if fr < 6:
            st = b.get_state(0)
            got = np.concatenate([st["gru_a_cond"], st["gru_b_cond"], st["lpc"]])
            assert np.array_equal(bits(got), bits(G["frame_cond"][fr])), fr
    st = b.get_state(0)
    assert np.array_equal(bits(st["gru_a_state"]), bits(G["final_gru_a_state"]))


@pytest.mark.parametrize("name", FIXTURES)
@pytest.mark.parametrize("B", [2, 300])
def test_constants_device_resident_paths(require_gpu, name, B):
    """lpcnet_batch_synthesize_frames: B = 2 overlaps the per-frame frame
    kernel with the sample kernel; B = 300 runs the chunked frame network
    (LPC ring over the chunk, rc2lpc per column) and multi-frame sample
    launches split at the stream's FEATURES_DELAY transition.  Every stream
    equals the per-frame host path; the fixture streams (placed at 0 and 5)
    equal the golden PCM, and two more streams equal the oracle."""
    G, c, variant = fixture(name)
    F = G["pcm"].shape[1]
    blob = blob_with(variant, c)
    allf = np.ascontiguousarray(np.stack([L.synthetic_features(s, F)[:, :20] for s in range(B)], 1))
    a = L.LPCNetBatch(B, 0, blob)
    ref = np.stack([a.synthesize(allf[f]) for f in range(F)], 0)
    b = L.LPCNetBatch(B, 0, blob)
    got = np.concatenate([_frames(b, allf, 0, 5), _frames(b, allf, 5, F)], 0)
    assert np.array_equal(got, ref)
    for si, s in enumerate(G["streams"]):
        if s < B:
            assert np.array_equal(got[:, s], G["pcm"][si]), s
    for s in (1, B - 1):
        exp = O.synth_stream(L.synthetic_model(1, variant), allf[:, s], variant, constants=c)
        assert np.array_equal(got[:, s], exp), s
    for s in (0, B - 1):
        sa, sb = a.get_state(s), b.get_state(s)
        for k in ("gru_a_state", "gru_b_state", "lpc", "gru_a_cond"):
            assert np.array_equal(bits(sa[k]), bits(sb[k])), (s, k)
        assert bytes(a.save_state(s)) == bytes(b.save_state(s)), s


def test_constants_setter_and_environment(require_gpu, monkeypatch):
    """lpcnet_batch_set_model_constants on a plain blob, and the LPCNET_*
    environment for the drop-in single-stream API (lpcnet_load_model of a
    blob without records), give the fixture; bad values are refused."""
    G, c, variant = fixture("streams_int8_g092_d3")
    blob = L.synthetic_model(1, variant)
    b = L.LPCNetBatch(2, 0, blob)
    assert b.info().features_delay == 2 and b.info().lpc_gamma == 1.0 and b.info().end2end == 0
    with pytest.raises(L.LPCNetError):
        b.set_model_constants(1.0, 5, False)
    b.set_model_constants(*c)
    out = np.stack([b.synthesize(G["features"][:, f, :20]) for f in range(G["pcm"].shape[1])], 1)
    assert np.array_equal(out, G["pcm"])
    G2, c2, _ = fixture("streams_int8_e2e_g09_d1")
    monkeypatch.setenv("LPCNET_LPC_GAMMA", repr(c2[0]))
    monkeypatch.setenv("LPCNET_FEATURES_DELAY", str(c2[1]))
    monkeypatch.setenv("LPCNET_END2END", str(c2[2]))
    net = L.LPCNet(blob)
    for fr in range(G2["pcm"].shape[1]):
        assert np.array_equal(net.synthesize(G2["features"][0, fr]), G2["pcm"][0, fr]), fr


@pytest.mark.parametrize("delay", [1, 2, 4])
@pytest.mark.parametrize("B", [300, 1100])
def test_deferred_lpc_ticks_match_eager_and_oracle(require_gpu, monkeypatch, delay, B):
    """One-frame ticks (lpcnet_batch_synthesize, > 128 streams: chunked frame
    network) with FEATURES_DELAY >= 1 push the frame's LPC into the ring
    after the sample kernel (deferred lpc_kernel); ticks on the batch's own
    pinned buffers (the chunk kernel's feature copy) and on caller arrays,
    interleaved with a multi-frame device-resident call and snapshots taken
    right after a tick, equal the eager order (LPCNET_LPC_EAGER=1) bit for
    bit on every stream, and the oracle on sampled streams."""
    c = (0.92, delay, 0)
    blob = blob_with(0, c)
    F = 9
    allf = np.ascontiguousarray(np.stack([L.synthetic_features(s, F)[:, :20] for s in range(B)], 1))

    def run():
        b = L.LPCNetBatch(B, 0, blob)
        hf = b.host_features()
        out, snaps = [], []
        for f in range(3):  # engine buffers (mapped features: the chunk kernel's copy feeds the LPC)
            np.copyto(hf, allf[f])
            out.append(np.array(b.synthesize_host()))
        snaps.append(bytes(b.save_state(B - 1)))
        out.extend(_frames(b, allf, 3, 6))  # multi-frame launch after deferred ticks
        for f in range(6, F):  # caller arrays (DMA-copied features)
            out.append(b.synthesize(allf[f]))
            snaps.append(bytes(b.save_state(0)))
        b.close()
        return np.stack(out, 0), snaps

    got, sg = run()
    monkeypatch.setenv("LPCNET_LPC_EAGER", "1")
    ref, sr = run()
    assert np.array_equal(got, ref)
    assert sg == sr
    for s in (0, B // 2, B - 1):
        exp = O.synth_stream(L.synthetic_model(1, 0), allf[:, s], 0, constants=c)
        assert np.array_equal(got[:, s], exp), s
