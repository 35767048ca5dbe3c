"""The drop-in API (include/lpcnet.h) shared across handles: every
LPCNetState bound to the same model on one device is a slot of one pool (one
device model, one work batch), and concurrent lpcnet_synthesize calls on
different handles coalesce into one launch (engine.cpp StatePool).  Each
handle must still produce exactly its own stream's reference PCM."""
import ctypes as C
import threading

import numpy as np
import pytest

import lpcnet_amd as L
import oracle_lib as O

pytestmark = pytest.mark.gpu


def pool_stats(net):
    la, rq, ns = C.c_long(0), C.c_long(0), C.c_int(0)
    assert L.lib.lpcnet_mi355x_pool_stats(C.c_void_p(net._st), C.byref(la), C.byref(rq), C.byref(ns)) == 0
    return la.value, rq.value, ns.value


def test_64_threads_share_one_pool_and_match_oracle(require_gpu):
    """64 threads, each lpcnet_create + lpcnet_load_model + 8 frames of
    lpcnet_synthesize on its own stream (features of stream id = thread id),
    all at once: every thread's PCM equals the oracle's; the 64 handles share
    one pool, and the calls coalesced (fewer launches than requests)."""
    T, F = 64, 8
    blob = L.synthetic_model(1, 0)
    feats = [L.synthetic_features(t, F)[:, :20] for t in range(T)]
    nets = [L.LPCNet(blob) for _ in range(T)]
    outs = [None] * T
    start = threading.Barrier(T)
    errors = []

    def run(t):
        try:
            start.wait()
            outs[t] = np.stack([nets[t].synthesize(feats[t][f]) for f in range(F)])
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=run, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=300)
    assert not errors, errors[:2]
    for t in range(T):
        assert np.array_equal(outs[t], O.synth_stream(blob, feats[t], 0)), t
    la, rq, ns = pool_stats(nets[0])
    assert ns == T and rq == T * F
    assert la < rq, (la, rq)  # coalesced
    for n in nets:
        n.close()


def test_handles_of_different_models_and_reset(require_gpu):
    """Handles on two different models use two pools; lpcnet_reset and
    lpcnet_init on a live handle reset only that handle's stream; a handle
    re-bound to another model keeps its stream state (lpcnet_load_model binds
    arrays only, lpcnet.c:202-210)."""
    a_blob, b_blob = L.synthetic_model(1, 0), L.synthetic_model(2, 0)
    f = L.synthetic_features(3, 6)[:, :20]
    na, nb, nc = L.LPCNet(a_blob), L.LPCNet(b_blob), L.LPCNet(a_blob)
    oa, ob = O.Oracle(a_blob, 0), O.Oracle(b_blob, 0)
    for k in range(4):
        assert np.array_equal(na.synthesize(f[k]), oa.synthesize(f[k]))
        assert np.array_equal(nb.synthesize(f[k]), ob.synthesize(f[k]))
        nc.synthesize(f[k])
    assert pool_stats(na)[2] == 2 and pool_stats(nb)[2] == 1
    nc.reset()
    oc = O.Oracle(a_blob, 0)
    assert np.array_equal(nc.synthesize(f[0]), oc.synthesize(f[0]))
    assert np.array_equal(na.synthesize(f[4]), oa.synthesize(f[4]))  # untouched by nc's reset
    # re-bind nb to model a: its state carries over
    nb.load_model(a_blob)
    assert pool_stats(na)[2] == 3
    # the same through the batch API: 4 frames on model b, the state moved
    # to a batch bound to model a
    xb = L.LPCNetBatch(1, 0, b_blob)
    for k in range(4):
        xb.synthesize(f[k][None])
    xa = L.LPCNetBatch(1, 0, a_blob)
    xa.restore_state(0, xb.save_state(0))
    assert np.array_equal(nb.synthesize(f[4]), xa.synthesize(f[4][None])[0])
    for n in (na, nb, nc):
        n.close()


@pytest.mark.parametrize("window,broadcast", [(50, 0), (0, 0), (200, 1)])
def test_pool_window_and_wakeups_match_oracle(require_gpu, monkeypatch, window, broadcast):
    """The pool's optional settings (read when a pool is created): gather
    window on or off, per-caller or broadcast wake-ups.  32 threads x 6
    frames, plus a save/restore on one handle half-way (slot I/O takes the
    pool while threads keep submitting): every stream equals the oracle's."""
    monkeypatch.setenv("LPCNET_POOL_WINDOW_US", str(window))
    monkeypatch.setenv("LPCNET_POOL_BROADCAST", str(broadcast))
    T, F = 32, 6
    blob = L.synthetic_model(20 + window + broadcast, 0)  # a model of its own: a fresh pool with these settings
    feats = [L.synthetic_features(t, F)[:, :20] for t in range(T)]
    nets = [L.LPCNet(blob) for _ in range(T)]
    monkeypatch.delenv("LPCNET_POOL_WINDOW_US")
    monkeypatch.delenv("LPCNET_POOL_BROADCAST")
    outs = [None] * T
    start = threading.Barrier(T)
    errors = []

    def run(t):
        try:
            start.wait()
            res = []
            for f in range(F):
                if t == 0 and f == F // 2:
                    snap = nets[0].save()
                    nets[0].restore(snap)
                res.append(nets[t].synthesize(feats[t][f]))
            outs[t] = np.stack(res)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=run, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=300)
    assert not errors, errors[:2]
    for t in range(T):
        assert np.array_equal(outs[t], O.synth_stream(blob, feats[t], 0)), t
    la, rq, ns = pool_stats(nets[0])
    assert ns == T and rq == T * F
    for n in nets:
        n.close()
