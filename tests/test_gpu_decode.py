"""The 1.6 kb/s decoder on the device (decode_kernel.hip: decode_packet,
lpcnet_dec.c:81-156, with perform_double_interp, common.c:36-65) feeding the
synthesis kernels (lpcnet_decode, lpcnet.c:310-319), against the CPU oracle:
decoded features bit-equal (through the PCM of every frame) and PCM
identical.  Parity of the decoder itself is unpinned by a reference build
(tests/test_decode_oracle.py says why); the engine and oracle are two
restatements checked against each other and against a numpy third."""
import threading

import numpy as np
import pytest

import lpcnet_amd as L
import oracle_lib as O

pytestmark = pytest.mark.gpu
BLOB = L.synthetic_model(1, L.VARIANT_INT8, codebooks=True)


def packets(nstreams, npk, seed=5):
    """[npk][nstreams][8] random packets; every interp id and vq_mid class occurs."""
    return np.random.default_rng(seed).integers(0, 256, size=(npk, nstreams, 8), dtype=np.uint8)


def oracle_decode(s, pk):
    o = O.Oracle(BLOB, 0)
    return np.stack([o.decode(bytes(pk[p, s])) for p in range(pk.shape[0])])  # [P][640]


@pytest.mark.parametrize("B", [1, 5])
def test_batch_decode_host_io_matches_oracle(require_gpu, B):
    P = 5
    pk = packets(B, P)
    b = L.LPCNetBatch(B, 0, BLOB)
    assert b.info().has_codebooks == 1
    got = np.stack([b.decode(pk[p]) for p in range(P)])  # [P][B][640]
    for s in range(B):
        assert np.array_equal(got[:, s], oracle_decode(s, pk)), s


@pytest.mark.parametrize("B,P", [(96, 10), (1024, 9)])
def test_batch_decode_frames_device_matches_oracle(require_gpu, B, P):
    """Device-resident packets -> PCM: 96 streams take the overlapped
    per-frame path, 1024 the chunked frame network and multi-frame sample
    launches; P spans two decode launches (8 packets each)."""
    pk = packets(B, P, seed=B)
    b = L.LPCNetBatch(B, 0, BLOB)
    d_pk = b.device_alloc(pk.nbytes)
    d_pcm = b.device_alloc(4 * P * B * 160 * 2)
    b.h2d(d_pk, pk)
    b.decode_frames(d_pk, d_pcm, P)
    b.sync()
    pcm = np.zeros((4 * P, B, 160), np.int16)
    b.d2h(pcm, d_pcm)
    for s in sorted({0, 1, B // 2, B - 1}):
        want = oracle_decode(s, pk).reshape(4 * P, 160)
        assert np.array_equal(pcm[:, s], want), s
    b.device_free(d_pk)
    b.device_free(d_pcm)


def test_decoder_state_carries_vq_mem(require_gpu):
    """vq_mem is part of a stream's saved state: a restored stream decodes
    its next packet as if never interrupted; a reset clears it as
    lpcnet_decoder_init does."""
    pk = packets(2, 4, seed=9)
    b = L.LPCNetBatch(2, 0, BLOB)
    b.decode(pk[0])
    b.decode(pk[1])
    snap = b.save_state(1)
    x = b.decode(pk[2])
    b.restore_state(1, snap)
    y = b.decode(pk[2])
    assert np.array_equal(x[1], y[1])
    b.reset()
    z = b.decode(pk[0])
    assert np.array_equal(z[0], oracle_decode(0, pk[:1])[0])


def test_dropin_decoder_threads_match_oracle(require_gpu):
    """lpcnet_decoder_create / lpcnet_decode on 8 threads at once (the
    requests coalesce in the pool): each decoder equals its oracle."""
    T, P = 8, 4
    pk = packets(T, P, seed=13)
    res = [None] * T
    start = threading.Barrier(T)
    decs = [L.LPCNetDecoder(BLOB) for _ in range(T)]

    def run(t):
        try:
            start.wait()
            res[t] = np.stack([decs[t].decode(bytes(pk[p, t])) for p in range(P)])
        except Exception as e:  # noqa: BLE001
            res[t] = e

    th = [threading.Thread(target=run, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=300)
    for t in range(T):
        assert isinstance(res[t], np.ndarray), res[t]
        assert np.array_equal(res[t], oracle_decode(t, pk)), t
    for d in decs:
        d.close()


def test_decoder_refuses_blob_without_codebooks(require_gpu):
    with pytest.raises(L.LPCNetError):
        L.LPCNetDecoder(L.synthetic_model(1, 0))
    b = L.LPCNetBatch(1, 0, L.synthetic_model(1, 0))
    assert b.info().has_codebooks == 0
    with pytest.raises(L.LPCNetError):
        b.decode(np.zeros((1, 8), np.uint8))


def test_decoder_reinit_keeps_model_and_resets_stream(require_gpu):
    """lpcnet_decoder_init on a live, bound decoder (the reference's way to
    reset one, lpcnet.c:290-295) resets its stream -- vq_mem included -- and
    keeps its model: decoding continues without a new load."""
    pk = packets(1, 4, seed=21)
    d = L.LPCNetDecoder(BLOB)
    first = np.stack([d.decode(bytes(pk[p, 0])) for p in range(2)])
    assert L.lib.lpcnet_decoder_init(d._st) == 0
    again = np.stack([d.decode(bytes(pk[p, 0])) for p in range(4)])
    want = oracle_decode(0, pk)
    assert np.array_equal(first, want[:2])
    assert np.array_equal(again, want)
    d.close()
