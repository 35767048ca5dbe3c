"""The reference-internal entry points the PLC drives (lpcnet_private.h:
126-132: lpcnet_synthesize_impl with preload, lpcnet_synthesize_tail_impl,
run_frame_network_deferred / _flush, lpcnet_reset_signal) and the PLC's
LPCNetState struct copies (lpcnet_plc.c:223,230), on the drop-in handle and
on the batch, against the CPU oracle (PCM identical every call, final GRU
states bit-equal).  The scenario replays the call sequences of
lpcnet_plc_update_causal / lpcnet_plc_conceal_causal (lpcnet_plc.c:188-337)
with PLC_SKIP_UPDATES defined (lpcnet_plc.c:40)."""
import threading

import numpy as np
import pytest

import lpcnet_amd as L
import oracle_lib as O

pytestmark = pytest.mark.gpu


def plc_scenario(net, ora, feats, seed):
    """Apply the same call sequence to an engine handle and the oracle;
    yield (what, engine PCM, oracle PCM) after every call that outputs."""
    rng = np.random.default_rng(seed)
    f = iter(feats)
    hist = np.zeros(160, np.int16)
    for _ in range(4):  # normal synthesis
        x = next(f)
        e, o = net.synthesize(x), ora.synthesize(x)
        yield "synthesize", e, o
        hist = o
    for _ in range(3):  # good packets: lpcnet_plc.c:272-276 (PLC_SKIP_UPDATES)
        x = next(f)
        net.frame_deferred(x)
        ora.frame_deferred(x)
    # a loss: conceal_causal (lpcnet_plc.c:293-320)
    net.frame_flush()
    ora.frame_flush()
    x = next(f)
    e = net.synthesize_impl(x, hist, 160)  # teacher-forced from the history (:308)
    o = ora.synthesize(x, 160, preload=hist)
    yield "impl preload 160", e, o
    tail = np.zeros(80, np.int16)
    yield "tail 80", net.synthesize_tail_impl(tail, 0), ora.synthesize_tail(tail, 0)  # :315
    x = next(f)
    e = net.synthesize_impl(x, np.zeros(80, np.int16), 0)  # :320
    o = ora.synthesize(x, 80)
    yield "impl 80", e, o
    # the blend after a loss (lpcnet_plc.c:221-231): speculate, roll back, teacher-force
    x = next(f)
    snap_e, snap_o = net.save(), ora.save()
    yield "speculate", net.synthesize_impl(x, np.zeros(80, np.int16), 0), ora.synthesize(x, 80)
    net.restore(snap_e)
    ora.restore(snap_o)
    pcm = rng.integers(-3000, 3000, 80).astype(np.int16)
    yield "impl preload 80", net.synthesize_impl(x, pcm, 80), ora.synthesize(x, 80, preload=pcm)
    # partial preload and partial N
    x = next(f)
    pcm = rng.integers(-3000, 3000, 121).astype(np.int16)
    yield "impl preload 37 of 121", net.synthesize_impl(x, pcm, 37), ora.synthesize(x, 121, preload=pcm[:37])
    # the non-blending branch (lpcnet_plc.c:233-236): reset the signal, go on
    net.reset_signal()
    ora.reset_signal()
    for _ in range(6):  # more deferred frames than the buffer holds (4)
        x = next(f)
        net.frame_deferred(x)
        ora.frame_deferred(x)
    net.frame_flush()
    ora.frame_flush()
    for _ in range(2):
        x = next(f)
        yield "synthesize after flush", net.synthesize(x), ora.synthesize(x)
    # a snapshot carries the deferred buffer
    x = next(f)
    net.frame_deferred(x)
    ora.frame_deferred(x)
    snap_e, snap_o = net.save(), ora.save()
    net.frame_flush()
    ora.frame_flush()
    net.restore(snap_e)
    ora.restore(snap_o)
    net.frame_flush()
    ora.frame_flush()
    x = next(f)
    yield "synthesize after restore", net.synthesize(x), ora.synthesize(x)


@pytest.mark.parametrize("variant,sat", [(0, False), (1, False), (0, True)])
def test_handle_plc_sequence_matches_oracle(require_gpu, variant, sat):
    blob = L.synthetic_model(1, variant, sat)
    feats = L.synthetic_features(11, 40)[:, :20]
    net, ora = L.LPCNet(blob), O.Oracle(blob, variant)
    n = 0
    for what, e, o in plc_scenario(net, ora, feats, 1):
        assert np.array_equal(e, o), f"{what}: first diff at {np.flatnonzero(e != o)[:5]}"
        n += 1
    assert n == 13
    net.close()


def test_handle_plc_sequences_concurrent(require_gpu):
    """16 threads, each replaying the scenario on its own handle (its own
    features): requests of the same shape coalesce across handles, the
    others run alone; every handle matches its own oracle."""
    T = 16
    blob = L.synthetic_model(1, 0)
    nets = [L.LPCNet(blob) for _ in range(T)]
    res = [None] * T
    start = threading.Barrier(T)

    def run(t):
        try:
            start.wait()
            feats = L.synthetic_features(100 + t, 40)[:, :20]
            ora = O.Oracle(blob, 0)
            res[t] = all(np.array_equal(e, o) for _, e, o in plc_scenario(nets[t], ora, feats, t))
        except Exception as e:  # noqa: BLE001
            res[t] = e

    th = [threading.Thread(target=run, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=300)
    assert all(r is True for r in res), res
    for n in nets:
        n.close()


@pytest.mark.parametrize("B", [3, 256])
def test_batch_tail_flush_reset_signal_match_oracle(require_gpu, B):
    """lpcnet_batch_synthesize_tail_impl, lpcnet_batch_run_frame_network in
    both modes and lpcnet_batch_reset_signal against per-stream oracles
    (streams 0, 1 and the last)."""
    blob = L.synthetic_model(1, 0)
    F = 10
    feats = np.stack([L.synthetic_features(s, F)[:, :20] for s in range(B)], 1)  # [F][B][20]
    b = L.LPCNetBatch(B, 0, blob)
    check = sorted({0, 1, B - 1})
    oras = {s: O.Oracle(blob, 0) for s in check}
    for fr in range(4):
        pcm = b.synthesize(feats[fr])
        for s in check:
            assert np.array_equal(pcm[s], oras[s].synthesize(feats[fr, s]))
    b.run_frame_network(feats[4], update_conditions=False)  # flush semantics
    for s in check:
        oras[s].frame_deferred(feats[4, s])
        oras[s].frame_flush()
    pcm = b.synthesize_tail_impl(np.zeros((B, 160), np.int16))
    for s in check:
        assert np.array_equal(pcm[s], oras[s].synthesize_tail(np.zeros(160, np.int16)))
    b.run_frame_network(feats[5], update_conditions=True)  # lpcnet_synthesize_impl(..., N = 0)
    for s in check:
        oras[s].synthesize(feats[5, s], 0)
    pre = np.random.default_rng(3).integers(-2000, 2000, (B, 100)).astype(np.int16)
    pcm = b.synthesize_tail_impl(pre, 50)
    for s in check:
        assert np.array_equal(pcm[s], oras[s].synthesize_tail(pre[s], 50))
    b.reset_signal(check[-1])
    oras[check[-1]].reset_signal()
    for fr in range(6, F):
        pcm = b.synthesize(feats[fr])
        for s in check:
            assert np.array_equal(pcm[s], oras[s].synthesize(feats[fr, s])), (fr, s)
    for s in check:
        st = b.get_state(s)
        a, bb = oras[s].state()
        assert np.array_equal(st["gru_a_state"].view(np.uint32), a.view(np.uint32))
        assert np.array_equal(st["gru_b_state"].view(np.uint32), bb.view(np.uint32))


def test_pool_create_load_synthesize_destroy_churn(require_gpu):
    """handles created, bound, used and destroyed concurrently on
    one model (pool reference counting under one lock): no crash, no leak of
    the pool (it is freed with its last handle and re-created), PCM right."""
    blob = L.synthetic_model(1, 0)
    feats = L.synthetic_features(9, 3)[:, :20]
    want = O.synth_stream(blob, feats, 0)
    T, R = 12, 6
    bad = []

    def run(t):
        try:
            for _ in range(R):
                n = L.LPCNet(blob)
                got = np.stack([n.synthesize(feats[k]) for k in range(3)])
                if not np.array_equal(got, want):
                    bad.append(t)
                n.close()
        except Exception as e:  # noqa: BLE001
            bad.append(e)

    th = [threading.Thread(target=run, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=300)
    assert not bad, bad[:3]
