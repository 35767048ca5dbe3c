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


@pytest.fixture(autouse=True)
def one_placement(request, monkeypatch):
    """These tests count handles per pool: pin every handle to device 0 (on a
    multi-GPU box the default placement spreads them over the devices)."""
    if "placement" not in request.node.name:
        monkeypatch.setenv("LPCNET_DEVICE", "0")


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


def _threads(T, fn):
    res = [None] * T
    start = threading.Barrier(T)

    def run(t):
        try:
            start.wait()
            res[t] = fn(t)
        except Exception as e:  # noqa: BLE001
            res[t] = e

    th = [threading.Thread(target=run, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=300)
    for r in res:
        assert not isinstance(r, Exception), r
    return res


def test_three_request_shapes_interleaved_match_oracle(require_gpu):
    """Three request shapes in flight on one pool at once -- full frames
    (N = 160), half frames (N = 80, the PLC's size) and frame-network-free
    tails (lpcnet_synthesize_tail_impl) -- so a combiner drains mixed shapes,
    runs one, and pushes the others back (oldest first): every
    handle equals its own oracle stream."""
    T, F = 24, 5
    blob = L.synthetic_model(31, 0)
    feats = [L.synthetic_features(t, F)[:, :20] for t in range(T)]
    nets = [L.LPCNet(blob) for _ in range(T)]

    def run(t):
        out = []
        for f in range(F):
            if t % 3 == 0:
                out.append(nets[t].synthesize(feats[t][f]))
            elif t % 3 == 1:
                out.append(nets[t].synthesize(feats[t][f], 80))
            else:
                out.append(nets[t].synthesize(feats[t][f], 80))
                out.append(nets[t].synthesize_tail_impl(np.zeros(80, np.int16)))
        return np.concatenate(out)

    got = _threads(T, run)
    for t in range(T):
        o = O.Oracle(blob, 0)
        want = []
        for f in range(F):
            if t % 3 == 0:
                want.append(o.synthesize(feats[t][f]))
            elif t % 3 == 1:
                want.append(o.synthesize(feats[t][f], 80))
            else:
                want.append(o.synthesize(feats[t][f], 80))
                want.append(o.synthesize_tail(np.zeros(80, np.int16)))
        assert np.array_equal(got[t], np.concatenate(want)), t
    for n in nets:
        n.close()


def test_placement_spreads_handles_and_matches_oracle(require_gpu, monkeypatch):
    """Drop-in placement (engine.cpp place_new_handle): with two placements
    of the one GPU (lpcnet_mi355x_set_placement([0, 0]), what
    LPCNET_DEVICES=0,0 sets), 16 handles split 8 / 8 by handle count, each
    placement runs its own pool, 16 threads at once, and every handle's PCM
    equals the oracle's; a destroyed handle frees its placement's count."""
    monkeypatch.delenv("LPCNET_DEVICE", raising=False)
    import gc
    gc.collect()
    L.set_placement([0, 0])
    try:
        T, F = 16, 5
        blob = L.synthetic_model(1, 0)
        feats = [L.synthetic_features(100 + t, F)[:, :20] for t in range(T)]
        nets = [L.LPCNet(blob) for _ in range(T)]
        places = [n.placement() for n in nets]
        assert sorted(p for _, p in places) == [0] * 8 + [1] * 8, places
        assert all(d == 0 for d, _ in places)
        got = _threads(T, lambda t: np.stack([nets[t].synthesize(feats[t][f]) for f in range(F)]))
        for t in range(T):
            assert np.array_equal(got[t], O.synth_stream(blob, feats[t], 0)), t
        by_place = {}
        for n, (_, p) in zip(nets, places):
            by_place.setdefault(p, pool_stats(n))
        assert by_place[0][2] == 8 and by_place[1][2] == 8, by_place
        assert by_place[0][1] == 8 * F and by_place[1][1] == 8 * F
        # least loaded: drop two handles of placement 1, the next two go there
        gone = [k for k, (_, p) in enumerate(places) if p == 1][:2]
        for k in gone:
            nets[k].close()
        extra = [L.LPCNet(blob) for _ in range(2)]
        assert [e.placement()[1] for e in extra] == [1, 1]
        f0 = feats[0][0]
        assert np.array_equal(extra[0].synthesize(f0), O.Oracle(blob, 0).synthesize(f0))
        for n in nets + extra:
            n.close()
    finally:
        gc.collect()
        L.set_placement([])
