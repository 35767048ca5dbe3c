"""Parity of the HIP path (through the C-ABI) with the golden fixtures made
from the reference's own kernels and with the CPU oracle.  Integer outputs
(PCM, excitation) must be identical; the pre-sampling logits and every float
state are compared bit for bit (tolerance 0 ulp: north_star asks for PCM
identity under identical kiss99 seeding, which requires bit-exact floats)."""
import os

import numpy as np
import pytest

import lpcnet_amd as L
import oracle_lib as O

pytestmark = pytest.mark.gpu
GOLD = O.GOLDEN


def feats(stream, nframes):
    return L.synthetic_features(stream, nframes)[:, :20]


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


@pytest.fixture(scope="module")
def blobs():
    return {"streams_int8": L.synthetic_model(1, 0), "streams_fp32": L.synthetic_model(1, 1),
            "streams_int8_sat": L.synthetic_model(1, 0, True)}


@pytest.mark.parametrize("name,kernel", [("streams_int8", 1), ("streams_fp32", 1), ("streams_int8_sat", 1),
                                         ("streams_int8", 4), ("streams_int8_sat", 4), ("streams_fp32", 4),
                                         ("streams_fp32", 5), ("streams_int8", 5), ("streams_int8_sat", 5),
                                         ("streams_int8", 0), ("streams_fp32", 0), ("streams_int8_sat", 0)])
def test_batch_matches_golden(require_gpu, blobs, name, kernel):
    """kernel 1: lockstep sample_kernel (quad_path 1 for int8 quad layouts,
    0 for fp32), 4: mf_kernel on the matrix cores, 5: fp_kernel (fp32),
    0: automatic (4 for non-saturating int8, 5 for fp32, 1 otherwise); a
    mode the model cannot run falls back to the lockstep kernel."""
    G = np.load(os.path.join(GOLD, name + ".npz"))
    streams = list(G["streams"])
    F = G["pcm"].shape[1]
    b = L.LPCNetBatch(len(streams), 0, blobs[name])
    b.set_kernel(kernel)
    if name == "streams_fp32":
        expect = {0: 5, 1: 0, 4: 0, 5: 5}[kernel]
    elif name.endswith("_sat"):
        expect = {0: 1, 1: 1, 4: 1, 5: 1}[kernel]
    else:
        expect = {0: 4, 1: 1, 4: 4, 5: 1}[kernel]
    assert b.info().quad_path == expect
    info = b.info()
    assert info.variant == int(G["variant"])
    if name.endswith("_sat"):
        assert info.may_saturate == 1
    b.set_trace(True)
    for fr in range(F):
        pcm = b.synthesize(G["features"][:, fr, :20])
        assert np.array_equal(pcm, G["pcm"][:, fr]), f"frame {fr}: first diff stream/sample " \
            f"{np.argwhere(pcm != G['pcm'][:, fr])[:3].tolist()}"
        if 2 <= fr < 6:
            lg, ex = b.get_trace(160)
            assert np.array_equal(ex[0], G["trace_exc"][fr - 2])
            assert np.array_equal(bits(lg[0]), bits(G["trace_logits"][fr - 2]))
        if fr < 6:
            st = b.get_state(0)
            got = np.concatenate([st["gru_a_cond"], st["gru_b_cond"], st["lpc"]])
            assert np.array_equal(bits(got), bits(G["frame_cond"][fr])), f"frame {fr} conditioning"
    st = b.get_state(0)
    assert np.array_equal(bits(st["gru_a_state"]), bits(G["final_gru_a_state"]))
    assert np.array_equal(bits(st["gru_b_state"]), bits(G["final_gru_b_state"]))


def test_single_stream_api_matches_golden(require_gpu, blobs):
    """lpcnet_create / lpcnet_load_model / lpcnet_synthesize (include/lpcnet.h)."""
    G = np.load(os.path.join(GOLD, "streams_int8.npz"))
    net = L.LPCNet(blobs["streams_int8"])
    for fr in range(G["pcm"].shape[1]):
        assert np.array_equal(net.synthesize(G["features"][0, fr]), G["pcm"][0, fr]), fr
    net.reset()
    assert np.array_equal(net.synthesize(G["features"][0, 0]), G["pcm"][0, 0])


@pytest.mark.parametrize("B,check,kernel", [(512, (0, 255, 511), 1), (1024, (0, 3, 517, 1023), 1),
                                            (1100, (1099, 1024, 5), 1), (1024, (0, 3, 517, 1023), 0),
                                            (1101, (1100, 1024, 5), 0), (300, (299, 7), 0),
                                            (513, (512, 1, 300), 4), (1030, (1029, 1027, 2), 4),
                                            (1024, (0, 511, 1023), 4), (4096, (0, 2047, 4095), 4)])
def test_large_batch_streams_match_oracle(require_gpu, blobs, B, check, kernel):
    """Lockstep kernel at 2 and 4 streams/workgroup, mf_kernel at 1, 2 and 4
    streams/workgroup, ragged last workgroups, against the oracle."""
    F = 5
    blob = blobs["streams_int8"]
    b = L.LPCNetBatch(B, 0, blob)
    b.set_kernel(kernel)
    allf = np.stack([feats(s, F) for s in range(B)], 1)  # [F][B][20]
    out = np.stack([b.synthesize(allf[f]) for f in range(F)], 1)  # [B][F][160]
    for s in check:
        ref = O.synth_stream(blob, allf[:, s], 0)
        assert np.array_equal(out[s], ref), s
    assert np.all(out[:, :2] == 0)  # FEATURES_DELAY silent frames
    assert np.abs(out[:, 2:]).mean() > 100


def test_matrix_core_kernel_edge_cases_at_bench_size(require_gpu, blobs, monkeypatch):
    """mf_kernel at 4 streams per workgroup (1026 streams: ragged last
    workgroup; LPCNET_MFW=0, the wide kernel would take this batch) through
    odd N, teacher forcing, a per-stream reset and the per-sample trace
    (logits bit for bit, excitation), against the oracle on streams of the
    first, a middle and the ragged workgroup; final GRU states."""
    monkeypatch.setenv("LPCNET_MFW", "0")
    B, F = 1026, 7
    blob = blobs["streams_int8"]
    allf = np.stack([feats(s, F) for s in range(B)], 1)
    check = (0, 1, 2, 3, 517, 1024, 1025)
    b = L.LPCNetBatch(B, 0, blob)
    b.set_kernel(4)
    assert b.info().quad_path == 4 and b.info().streams_per_workgroup == 4
    b.set_trace(True)
    refs = {s: O.Oracle(blob, 0) for s in check}
    t = np.arange(160)
    for f in range(F):
        if f == 5:
            b.reset(2)
            refs[2] = O.Oracle(blob, 0)
        pre, n = (77, 160) if f == 4 else (0, 81 if f == 3 else 160)
        if pre:
            teacher = np.stack([(2500 * np.sin(0.03 * (s % 7 + 1) * t)).astype(np.int16) for s in range(B)])
            out = b.synthesize_impl(allf[f], teacher, pre)
        else:
            out = b.synthesize(allf[f], n)
        lg, ex = b.get_trace(n)
        for s in check:
            exp, elg, eex, _ = refs[s].synthesize(allf[f, s], n, preload=teacher[s][:pre] if pre else None, trace=True)
            assert np.array_equal(out[s], exp), (f, s)
            if f >= 2 and not (s == 2 and f >= 5):  # silent frames after the reset: no trace
                assert np.array_equal(ex[s, pre:], eex[pre:]), (f, s)
                assert np.array_equal(bits(lg[s, pre:]), bits(elg[pre:])), (f, s)
    for s in check:
        a, g = refs[s].state()
        st = b.get_state(s)
        assert np.array_equal(bits(st["gru_a_state"]), bits(a)), s
        assert np.array_equal(bits(st["gru_b_state"]), bits(g)), s


@pytest.mark.parametrize("env", ["LPCNET_MF_EXACT", "LPCNET_MF_ZR_BOUND=0.05", "LPCNET_MF_ZR_BOUND=1.5", "LPCNET_FC_EXACT"])
@pytest.mark.parametrize("B,check", [(1030, (0, 1, 2, 3, 517, 1029)), (70, (0, 37, 69))])
@pytest.mark.parametrize("mf2", ["0", "1"])
def test_matrix_core_range_paths_match_oracle(require_gpu, blobs, monkeypatch, env, B, check, mf2):
    """mf_kernel's GRU_A elementwise has a select-free form for workgroups
    whose conditioning and states lie within the host's range bounds, and the
    exact form with x86's out-of-range/NaN selects otherwise.  Force the exact
    form everywhere, or lower the z/r bound so workgroups split between the
    two (the bound is a launch-time property of each workgroup's streams):
    PCM and final GRU_A states against the oracle."""
    name, _, val = env.partition("=")
    monkeypatch.setenv(name, val or "1")
    monkeypatch.setenv("LPCNET_MF2", mf2)  # mf_kernel / mf2_kernel
    F = 6
    blob = blobs["streams_int8"]
    b = L.LPCNetBatch(B, 0, blob)
    b.set_kernel(4)
    allf = np.stack([feats(s, F) for s in range(B)], 1)
    out = np.stack([b.synthesize(allf[f]) for f in range(F)], 1)
    for s in check:
        o = O.Oracle(blob, 0)
        exp = np.stack([o.synthesize(allf[f, s]) for f in range(F)])
        assert np.array_equal(out[s], exp), s
        a, _ = o.state()
        assert np.array_equal(bits(b.get_state(s)["gru_a_state"]), bits(a)), s


@pytest.mark.parametrize("B,check", [(1, (0,)), (70, (0, 37, 69))])
def test_fp32_latency_kernel_matches_oracle(require_gpu, blobs, B, check):
    """fp_kernel (one stream per workgroup) against the fp32 oracle, with a
    partial frame (N = 80) and a per-stream reset in the middle."""
    F = 7
    blob = blobs["streams_fp32"]
    b = L.LPCNetBatch(B, 0, blob)
    b.set_kernel(5)
    assert b.info().quad_path == 5
    allf = np.stack([feats(s, F) for s in range(B)], 1)
    refs = {s: O.Oracle(blob, 1) for s in check}
    for f in range(F):
        if f == 5:
            b.reset(check[-1])
            refs[check[-1]] = O.Oracle(blob, 1)
        n = 80 if f == 4 else 160
        out = b.synthesize(allf[f], n)
        for s in check:
            assert np.array_equal(out[s], refs[s].synthesize(allf[f, s], n)), (f, s)
        if f == 3:
            assert np.abs(out.astype(np.float64)).mean() > 100


def _frames(b, allf, f0, f1):
    """lpcnet_batch_synthesize_frames over frames f0..f1-1 -> [F][B][160]"""
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


@pytest.mark.parametrize("B,name", [(64, "streams_int8"), (1, "streams_int8"), (1, "streams_fp32"),
                                    (3, "streams_fp32"), (100, "streams_fp32"), (128, "streams_int8"),
                                    (129, "streams_int8"), (64, "streams_int8_sat")])
def test_device_resident_frames_equal_host_path(require_gpu, blobs, B, name):
    """lpcnet_batch_synthesize_frames (pipelined host LPC; up to
    OVERLAP_MAX_STREAMS = 128 streams the frame kernel of frame f+1 runs beside
    the sample kernel of frame f, outputs double-buffered) == frame-by-frame
    host API, including the frame conditioning left in the stream state, and
    mixed with single-frame calls; B = 1 also against the oracle."""
    F = 9
    blob = blobs[name]
    variant = 1 if name == "streams_fp32" else 0
    allf = np.ascontiguousarray(np.stack([feats(s, F) for s in range(B)], 1))
    a = L.LPCNetBatch(B, 0, blob)
    ref = np.stack([a.synthesize(allf[f]) for f in range(F)], 0)
    b = L.LPCNetBatch(B, 0, blob)
    got = np.concatenate([_frames(b, allf, 0, 5), b.synthesize(allf[5])[None], _frames(b, allf, 6, F)], 0)
    assert np.array_equal(got, ref)
    for s in (0, B - 1):
        sa, sb = a.get_state(s), b.get_state(s)
        for k in ("gru_a_state", "gru_b_state", "gru_a_cond", "gru_b_cond", "lpc"):
            assert np.array_equal(bits(sa[k]), bits(sb[k])), (s, k)
    if B == 1:
        assert np.array_equal(got[:, 0], O.synth_stream(blob, allf[:, 0], variant))


def test_partial_frame_and_reset_stream(require_gpu, blobs):
    """N < 160 (lpcnet_synthesize with N=80) and a per-stream reset mid-run."""
    blob = blobs["streams_int8"]
    B, F = 4, 8
    allf = np.stack([feats(s, F) for s in range(B)], 1)
    b = L.LPCNetBatch(B, 0, blob)
    ref = [O.Oracle(blob, 0) for _ in range(B)]
    for f in range(F):
        if f == 4:
            b.reset(2)
            ref[2] = O.Oracle(blob, 0)
        n = 80 if f % 2 else 160
        out = b.synthesize(allf[f], n)
        for s in range(B):
            assert np.array_equal(out[s], ref[s].synthesize(allf[f, s], n)), (f, s)


def test_rejects_bad_blob(require_gpu, blobs):
    b = L.LPCNetBatch(2, 0)
    with pytest.raises(L.LPCNetError):
        b.load_model(blobs["streams_int8"][:-64])
    with pytest.raises(L.LPCNetError):
        b.synthesize(np.zeros((2, 20), np.float32))  # no model bound


def test_full_size_properties(require_gpu, blobs):
    """At the bench size (1024 streams): determinism across runs, stream
    independence (permuting the batch permutes the output), sane PCM."""
    B, F = 1024, 4
    blob = blobs["streams_int8"]
    allf = np.stack([feats(s, F) for s in range(B)], 1)
    perm = np.random.default_rng(3).permutation(B)
    b1 = L.LPCNetBatch(B, 0, blob)
    o1 = np.stack([b1.synthesize(allf[f]) for f in range(F)], 1)
    b2 = L.LPCNetBatch(B, 0, blob)
    o2 = np.stack([b2.synthesize(allf[f][perm]) for f in range(F)], 1)
    assert np.array_equal(o1[perm], o2)
    b1.reset()
    o3 = np.stack([b1.synthesize(allf[f]) for f in range(F)], 1)
    assert np.array_equal(o1, o3)
    assert np.abs(o1[:, 2:].astype(np.float64)).mean() > 100


@pytest.mark.parametrize("kernel,variant", [(1, 0), (4, 0), (5, 1), (1, 1)])
def test_preload_teacher_forcing_matches_oracle(require_gpu, blobs, kernel, variant):
    """lpcnet_synthesize_impl with preload (lpcnet.c:256-259, the PLC entry)."""
    blob = blobs["streams_fp32" if variant else "streams_int8"]
    B, F = 3, 9
    allf = np.stack([feats(s, F) for s in range(B)], 1)
    b = L.LPCNetBatch(B, 0, blob)
    b.set_kernel(kernel)
    refs = [O.Oracle(blob, variant) for _ in range(B)]
    t = np.arange(160)
    for f in range(F):
        if f in (4, 6):
            pre = 80 if f == 4 else 160
            teacher = np.stack([(3000 * np.sin(0.05 * (s + 1) * t)).astype(np.int16) for s in range(B)])
            out = b.synthesize_impl(allf[f], teacher, pre)
            for s in range(B):
                exp = refs[s].synthesize(allf[f, s], 160, preload=teacher[s][:pre] if pre < 160 else teacher[s])
                if pre < 160:
                    exp = np.concatenate([teacher[s][:pre], exp[pre:]])
                assert np.array_equal(out[s], exp), (f, s)
        else:
            out = b.synthesize(allf[f])
            for s in range(B):
                assert np.array_equal(out[s], refs[s].synthesize(allf[f, s])), (f, s)


def test_frame_network_only_flush(require_gpu, blobs):
    """N == 0: frame network only (run_frame_network_flush, lpcnet.c:134-144)."""
    blob = blobs["streams_int8"]
    B, F = 2, 6
    allf = np.stack([feats(s, F) for s in range(B)], 1)
    b = L.LPCNetBatch(B, 0, blob)
    refs = [O.Oracle(blob, 0) for _ in range(B)]
    for f in range(F):
        if f in (1, 3):
            b.frame_only(allf[f])
            for s in range(B):
                refs[s].synthesize(allf[f, s], 0)
        else:
            out = b.synthesize(allf[f])
            for s in range(B):
                assert np.array_equal(out[s], refs[s].synthesize(allf[f, s])), (f, s)


def test_state_save_restore_rollback(require_gpu, blobs):
    """Speculate-and-roll-back as lpcnet_plc.c:223-231 does with struct copies."""
    blob = blobs["streams_int8"]
    B, F = 2, 8
    allf = np.stack([feats(s, F) for s in range(B)], 1)
    b = L.LPCNetBatch(B, 0, blob)
    for f in range(4):
        b.synthesize(allf[f])
    snap = b.save_state(1)
    first = np.stack([b.synthesize(allf[f]) for f in range(4, 6)])
    b.restore_state(1, snap)
    second = np.stack([b.synthesize(allf[f]) for f in range(4, 6)])
    assert np.array_equal(first[:, 1], second[:, 1])


def test_restore_refuses_out_of_range_gru_state(require_gpu, blobs):
    """A snapshot whose GRU state lies outside [-2, 2] cannot come from the
    recurrence (states are convex combinations of tanh outputs) and would
    break the int8 state quantiser's range: restore refuses it.  NaN states
    (what NaN features produce) are accepted."""
    import struct
    blob = blobs["streams_int8"]
    B, F = 2, 5
    allf = np.stack([feats(s, F) for s in range(B)], 1)
    b = L.LPCNetBatch(B, 0, blob)
    for f in range(4):
        b.synthesize(allf[f])
    snap = bytes(b.save_state(0))
    off = snap.find(b.get_state(0)["gru_a_state"].tobytes())
    assert off >= 0
    bad = bytearray(snap)
    struct.pack_into("<f", bad, off + 4 * 5, 3.0)
    with pytest.raises(L.LPCNetError):
        b.restore_state(0, bytes(bad))
    nan = bytearray(snap)
    struct.pack_into("<f", nan, off, float("nan"))
    b.restore_state(0, bytes(nan))
    b.restore_state(0, snap)
    ref = L.LPCNetBatch(B, 0, blob)
    for f in range(4):
        ref.synthesize(allf[f])
    assert np.array_equal(b.synthesize(allf[4]), ref.synthesize(allf[4]))


@pytest.mark.parametrize("mf2", ["0", "1"])
def test_walk_exact_form_for_states_outside_the_bound(require_gpu, blobs, monkeypatch, mf2):
    """The dual-FC walk takes its select-free tanh only when the model's node
    sums are bounded (SampleArgs::fc_fin) and every GRU_B state of the
    workgroup lies within [-2, 2] at launch.  A restored NaN GRU_B state
    (accepted by restore) must send that workgroup through the exact x86
    form: the same PCM as with the exact form forced (LPCNET_FC_EXACT)."""
    import struct
    monkeypatch.setenv("LPCNET_MF2", mf2)
    blob = blobs["streams_int8"]
    B, F = 2048 if mf2 == "1" else 3, 7
    allf = np.stack([feats(s % 3, F) for s in range(B)], 1)
    outs = []
    for exact in ("0", "1"):
        monkeypatch.setenv("LPCNET_FC_EXACT", exact)
        b = L.LPCNetBatch(B, 0, blob)
        b.set_kernel(4)
        for f in range(4):
            b.synthesize(allf[f])
        snap = bytearray(b.save_state(1))
        off = bytes(snap).find(b.get_state(1)["gru_b_state"].tobytes())
        assert off >= 0
        struct.pack_into("<f", snap, off + 4 * 3, float("nan"))
        b.restore_state(1, bytes(snap))
        outs.append(np.stack([b.synthesize(allf[f]) for f in range(4, F)], 1))
        b.close()
    assert np.array_equal(outs[0], outs[1])


def test_restore_refuses_out_of_range_last_exc(require_gpu, blobs):
    """last_exc indexes the 256-row embedding tables: a snapshot with
    last_exc outside [0, 255] is refused (at 512 streams mf_kernel<2> turns
    it into a byte offset of the gather); the spin-limit setter clamps huge
    bounds instead of letting the poll counter overflow."""
    import struct
    blob = blobs["streams_int8"]
    B, F = 512, 4
    allf = np.stack([feats(s, F) for s in range(B)], 1)
    b = L.LPCNetBatch(B, 0, blob)
    assert b.info().streams_per_workgroup == 2
    for f in range(3):
        b.synthesize(allf[f])
    snap = bytes(b.save_state(7))
    # StreamState ends ..., deemph_mem, last_exc, frame_count (= 3 now), rng[4], vq_mem[18] (0), pad[3]
    i32 = lambda o: struct.unpack_from("<i", snap, o)[0]  # noqa: E731
    offs = [o for o in range(len(snap) - 160, len(snap) - 8, 4)
            if i32(o + 4) == 3 and 0 <= i32(o) <= 255 and snap[o + 24:o + 24 + 72] == bytes(72)]
    assert len(offs) == 1, offs
    off = offs[0]
    for v in (256, -1, 1 << 20):
        bad = bytearray(snap)
        struct.pack_into("<i", bad, off, v)
        with pytest.raises(L.LPCNetError, match="last_exc"):
            b.restore_state(7, bytes(bad))
    b.restore_state(7, snap)
    b.set_spin_limit(2 ** 31 - 1)
    ref = L.LPCNetBatch(B, 0, blob)
    for f in range(3):
        ref.synthesize(allf[f])
    assert np.array_equal(b.synthesize(allf[3]), ref.synthesize(allf[3]))


def test_8192_streams_one_gpu_match_oracle(require_gpu, blobs):
    """BASELINE configs[4]'s total stream count on one GPU: LPCNetBatch(8192)
    through the device-resident multi-frame path (mfw_kernel: 1024
    workgroups of two 4-stream groups, chunked frame network), against the
    CPU oracle on two streams of every 1024-stream shard (PCM and final GRU
    states bit for bit), and shard 3 run alone as a 1024-stream batch gives
    the same PCM for its streams."""
    B, F = 8192, 8
    blob = blobs["streams_int8"]
    allf = np.ascontiguousarray(np.stack([feats(s, F) for s in range(B)], 1))
    b = L.LPCNetBatch(B, 0, blob)
    assert b.info().quad_path == 7 and b.info().streams_per_workgroup == 8  # mfw_kernel, two groups
    b.reset_timers(1)
    got = np.concatenate([_frames(b, allf, 0, 2), _frames(b, allf, 2, F)], 0)
    assert b.kernel_frames(0) == F and b.kernel_ms(0)[1] == 3  # 2 single-frame launches + one of 6
    assert np.abs(got[2:].astype(np.float64)).mean() > 100
    for shard in range(8):
        for sid in (1024 * shard + (37 * shard) % 1024, 1024 * shard + 1023 - shard):
            o = O.Oracle(blob, 0)
            exp = np.stack([o.synthesize(allf[f, sid]) for f in range(F)])
            assert np.array_equal(got[:, sid], exp), sid
            a, g = o.state()
            st = b.get_state(sid)
            assert np.array_equal(bits(st["gru_a_state"]), bits(a)), sid
            assert np.array_equal(bits(st["gru_b_state"]), bits(g)), sid
    b.close()
    c = L.LPCNetBatch(1024, 0, blob)
    alone = np.concatenate([_frames(c, allf[:, 3072:4096], 0, 2), _frames(c, allf[:, 3072:4096], 2, F)], 0)
    assert np.array_equal(alone, got[:, 3072:4096])


@pytest.mark.parametrize("B", [9, 70, 1030, 2048])
def test_mf2_kernel_equals_mf_kernel(require_gpu, blobs, monkeypatch, B):
    """mf2_kernel (two 4-stream groups per workgroup, half a sample apart;
    LPCNET_MF2=1 forces it at any batch) against mf_kernel (LPCNET_MF2=0):
    the PCM and the complete stream state byte for byte, every stream,
    through the per-frame host path (with a partial frame, N = 81, and a
    per-stream reset) and the device-resident multi-frame path (runs that
    start inside the FEATURES_DELAY frames and span chunk boundaries);
    ragged last workgroups at 9 and 70 streams.  Preload and trace calls fall
    back to mf_kernel on the same batch.  Stream 0 against the oracle."""
    F = 40
    blob = blobs["streams_int8"]
    allf = np.ascontiguousarray(np.stack([feats(s, F) for s in range(B)], 1))
    outs, states = [], []
    monkeypatch.setenv("LPCNET_MFW", "0")  # mf2_kernel itself, not the wide kernel that replaces it
    for mf2 in ("0", "1"):
        monkeypatch.setenv("LPCNET_MF2", mf2)
        b = L.LPCNetBatch(B, 0, blob)
        assert b.info().quad_path == (6 if mf2 == "1" else 4)
        parts = [np.stack([b.synthesize(allf[f]) for f in range(3)])]
        parts.append(np.pad(b.synthesize(allf[3], 81), ((0, 0), (0, 79)))[None])
        b.reset(B - 1)
        parts.append(_frames(b, allf, 4, 7))
        parts.append(_frames(b, allf, 7, F))
        outs.append(np.concatenate(parts, 0))
        states.append([bytes(b.save_state(s)) for s in range(B)])
        b.close()
    assert np.abs(outs[0][8:].astype(np.float64)).mean() > 100
    bad = np.nonzero((outs[1] != outs[0]).any(axis=2))
    assert not len(bad[0]), list(zip(bad[0][:8], bad[1][:8]))
    badst = [s for s in range(B) if states[1][s] != states[0][s]]
    assert not badst, badst[:8]
    o = O.Oracle(blob, 0)
    ref = [o.synthesize(allf[f, 0]) for f in range(3)] + [np.pad(o.synthesize(allf[3, 0], 81), (0, 79))]
    ref += [o.synthesize(allf[f, 0]) for f in range(4, F)]
    assert np.array_equal(outs[1][:, 0], np.stack(ref))


@pytest.mark.parametrize("mfw", ["0", "1"])
def test_mf2_batch_falls_back_for_preload_and_trace(require_gpu, blobs, monkeypatch, mfw):
    """A 2048-stream batch (mf2_kernel, or the mfw_kernel that replaces it by
    default) takes mf_kernel for a teacher-forced call and for a traced call:
    PCM, logits and excitation against the oracle."""
    monkeypatch.delenv("LPCNET_MF2", raising=False)
    monkeypatch.setenv("LPCNET_MFW", mfw)
    B, F = 2048, 5
    blob = blobs["streams_int8"]
    allf = np.stack([feats(s, F) for s in range(B)], 1)
    b = L.LPCNetBatch(B, 0, blob)
    assert b.info().quad_path == (7 if mfw == "1" else 6)
    check = (0, 1500, 2047)
    refs = {s: O.Oracle(blob, 0) for s in check}
    t = np.arange(160)
    for f in range(F):
        if f == 3:
            teacher = np.stack([(2000 * np.sin(0.02 * (s % 5 + 1) * t)).astype(np.int16) for s in range(B)])
            out = b.synthesize_impl(allf[f], teacher, 60)
            for s in check:
                exp = refs[s].synthesize(allf[f, s], 160, preload=teacher[s][:60])
                assert np.array_equal(out[s], exp), (f, s)
        elif f == 4:
            b.set_trace(True)
            out = b.synthesize(allf[f])
            lg, ex = b.get_trace(160)
            for s in check:
                exp, elg, eex, _ = refs[s].synthesize(allf[f, s], 160, trace=True)
                assert np.array_equal(out[s], exp) and np.array_equal(ex[s], eex), (f, s)
                assert np.array_equal(bits(lg[s]), bits(elg)), (f, s)
        else:
            out = b.synthesize(allf[f])
            for s in check:
                assert np.array_equal(out[s], refs[s].synthesize(allf[f, s])), (f, s)


CHECK256 = (0, 1, 128, 254, 255)


def test_batch256_auto_kernel_matches_oracle(require_gpu, blobs):
    """BASELINE configs[2]: 256 streams on the automatic kernel (mf_kernel<1>,
    256 workgroups; one-stream frame-kernel workgroups) through
    lpcnet_batch_synthesize, against the oracle on streams 0, 1, 128, 254,
    255: PCM, the 8 traced pre-sampling logits bit for bit, the excitation,
    and the final GRU states; then lpcnet_batch_synthesize_frames over the
    same frames gives the same PCM for every stream."""
    B, F = 256, 6
    blob = blobs["streams_int8"]
    allf = np.ascontiguousarray(np.stack([feats(s, F) for s in range(B)], 1))
    b = L.LPCNetBatch(B, 0, blob)
    info = b.info()
    assert info.quad_path == 4 and info.streams_per_workgroup == 1
    b.set_trace(True)
    refs = {s: O.Oracle(blob, 0) for s in CHECK256}
    outs = []
    for f in range(F):
        out = b.synthesize(allf[f])
        outs.append(out)
        lg, ex = b.get_trace(160)
        for s in CHECK256:
            exp, elg, eex, _ = refs[s].synthesize(allf[f, s], 160, trace=True)
            assert np.array_equal(out[s], exp), (f, s)
            if f >= 2:
                assert np.array_equal(ex[s], eex), (f, s)
                assert np.array_equal(bits(lg[s]), bits(elg)), (f, s)
    for s in CHECK256:
        a, g = refs[s].state()
        st = b.get_state(s)
        assert np.array_equal(bits(st["gru_a_state"]), bits(a)), s
        assert np.array_equal(bits(st["gru_b_state"]), bits(g)), s
    assert np.abs(np.stack(outs)[2:].astype(np.float64)).mean() > 100
    c = L.LPCNetBatch(B, 0, blob)
    got = _frames(c, allf, 0, F)
    assert np.array_equal(got, np.stack(outs))


@pytest.mark.parametrize("B,name", [(129, "streams_int8"), (256, "streams_int8"), (1024, "streams_int8"),
                                    (2050, "streams_int8"), (200, "streams_fp32")])
def test_chunked_frame_network_equals_per_frame(require_gpu, blobs, B, name):
    """Above 128 streams lpcnet_batch_synthesize_frames runs the frame network
    of up to 32 frames in one chunk_kernel launch (f32 matrix cores).  Runs of
    37 frames (chunks of 32 and 5), 20 and 24 frames (at 1024 streams the 20 x
    4 and 24 x 4 column layouts), then 3 frames (below CHUNK_MIN_FRAMES:
    per-frame kernel) must give the PCM and the complete stream state (conv
    memories, LPC ring, frame_count, conditioning, GRU states, RNG) of the
    per-frame frame kernel, byte for byte, every stream."""
    F = 84
    blob = blobs[name]
    allf = np.ascontiguousarray(np.stack([feats(s, F) for s in range(B)], 1))
    outs, states = [], []
    for chunking in (False, True):
        b = L.LPCNetBatch(B, 0, blob)
        b.set_frame_chunking(chunking)
        got = np.concatenate([_frames(b, allf, 0, 37), _frames(b, allf, 37, 57), _frames(b, allf, 57, 81),
                              _frames(b, allf, 81, F)], 0)
        outs.append(got)
        states.append([bytes(b.save_state(s)) for s in range(B)])
        b.close()
    assert np.abs(outs[0][2:].astype(np.float64)).mean() > 100
    assert np.array_equal(outs[1], outs[0])
    bad = [s for s in range(B) if states[1][s] != states[0][s]]
    assert not bad, bad[:8]


@pytest.mark.parametrize("B,mfw", [(1, "0"), (2, "0"), (70, "0"), (256, "0"), (1030, "0"), (1030, "1"), (2100, "1")])
def test_multi_frame_sample_launches_match_per_frame(require_gpu, blobs, monkeypatch, B, mfw):
    """lpcnet_batch_synthesize_frames on the matrix-core kernel launches the
    sample kernel once per chunk of frames (SampleArgs::nframes), carrying the
    states in registers across frames.  Against the per-frame launches
    (LPCNET_NO_MULTIFRAME) over runs that start at a reset (the FEATURES_DELAY
    frames go to single-frame launches), follow a per-stream reset and a
    state restore mid-run, and span chunk boundaries: the PCM and the complete
    stream state byte for byte, every stream; stream 0 also against the
    oracle.  The timers count one launch per multi-frame run.  mfw = 1: the
    same on the wide kernel (two groups per workgroup at 1030 and 2100)."""
    monkeypatch.setenv("LPCNET_MFW", mfw)
    F = 44
    blob = blobs["streams_int8"]
    allf = np.ascontiguousarray(np.stack([feats(s, F) for s in range(B)], 1))
    runs = [(0, 6), (6, 40), (40, F)]
    outs, states = [], []
    for multi in (False, True):
        if multi:
            monkeypatch.delenv("LPCNET_NO_MULTIFRAME", raising=False)
        else:
            monkeypatch.setenv("LPCNET_NO_MULTIFRAME", "1")
        b = L.LPCNetBatch(B, 0, blob)
        assert b.info().quad_path == (7 if mfw == "1" else 4)
        parts = []
        for i, (f0, f1) in enumerate(runs):
            if i == 1:
                b.reset(B - 1)
            if i == 2:
                snap = bytes(b.save_state(0))
                b.restore_state(0, snap)
            b.reset_timers(1)
            parts.append(_frames(b, allf, f0, f1))
            if multi and i == 1:
                ms, n = b.kernel_ms(0)
                # frames 6..37: two single-frame launches (stream B-1 reset) + one of 30;
                # frames 38..39: below CHUNK_MIN_FRAMES, per frame
                assert b.kernel_frames(0) == 34 and n == 5, (b.kernel_frames(0), n)
        outs.append(np.concatenate(parts, 0))
        states.append([bytes(b.save_state(s)) for s in range(B)])
        b.close()
    assert np.abs(outs[0][3:].astype(np.float64)).mean() > 100
    bad = np.nonzero((outs[1] != outs[0]).any(axis=2))
    assert not len(bad[0]), list(zip(bad[0][:8], bad[1][:8]))
    badst = [s for s in range(B) if states[1][s] != states[0][s]]
    assert not badst, badst[:8]
    if B <= 2:
        o = O.Oracle(blob, 0)
        ref = []
        for f in range(F):
            if f == 6 and B == 1:
                o = O.Oracle(blob, 0)  # stream B-1 = 0 was reset
            ref.append(o.synthesize(allf[f, 0]))
        ref = np.stack(ref)
        assert np.array_equal(outs[1][:, 0], ref)


@pytest.mark.parametrize("B,name", [(1, "streams_int8"), (1, "streams_fp32"), (64, "streams_int8"),
                                    (300, "streams_int8")])
def test_unsynced_frames_then_single_frame(require_gpu, blobs, B, name):
    """lpcnet_batch_synthesize_frames returns with frames still queued (an odd
    count leaves the last one reading pinned LPC slot 0); a single-frame call
    made right after, with no lpcnet_batch_sync, must not disturb them."""
    F = 7
    blob = blobs[name]
    allf = np.ascontiguousarray(np.stack([feats(s, F) for s in range(B)], 1))
    a = L.LPCNetBatch(B, 0, blob)
    ref = np.stack([a.synthesize(allf[f]) for f in range(F)], 0)
    b = L.LPCNetBatch(B, 0, blob)
    part = np.ascontiguousarray(allf[:5])
    df = b.device_alloc(part.nbytes)
    dp = b.device_alloc(5 * B * 160 * 2)
    b.h2d(df, part)
    b.synthesize_frames(part, df, dp, 5)
    out5 = b.synthesize(allf[5])            # no sync in between
    out6 = b.synthesize(allf[6])
    got = np.zeros((5, B, 160), np.int16)
    b.d2h(got, dp)
    b.device_free(df)
    b.device_free(dp)
    assert np.array_equal(got, ref[:5])
    assert np.array_equal(out5, ref[5]) and np.array_equal(out6, ref[6])


def test_device_abort_is_reported_not_silent(require_gpu, blobs):
    """fp_kernel's LDS flag waits are bounded; with the bound forced to one
    poll every launch aborts, and the call must fail (-1, last_error) instead
    of returning PCM.  The default bound then synthesises correctly again."""
    blob = blobs["streams_fp32"]
    B, F = 2, 4
    allf = np.ascontiguousarray(np.stack([feats(s, F) for s in range(B)], 1))
    b = L.LPCNetBatch(B, 0, blob)
    assert b.info().quad_path == 5
    for f in range(3):
        b.synthesize(allf[f])  # frames 0-2: frame 2 is the first non-silent one
    b.set_spin_limit(1)
    with pytest.raises(L.LPCNetError, match="spin limit"):
        b.synthesize(allf[3])
    # the queued path reports at the sync
    df = b.device_alloc(allf.nbytes)
    dp = b.device_alloc(F * B * 160 * 2)
    b.h2d(df, allf)
    b.synthesize_frames(allf, df, dp, F)
    with pytest.raises(L.LPCNetError, match="spin limit"):
        b.sync()
    b.device_free(df)
    b.device_free(dp)
    b.set_spin_limit(0)
    b.reset()
    refs = [O.Oracle(blob, 1) for _ in range(B)]
    for f in range(F):
        out = b.synthesize(allf[f])
        for s in range(B):
            assert np.array_equal(out[s], refs[s].synthesize(allf[f, s])), (f, s)


def test_drop_in_api_error_behaviour(require_gpu, blobs):
    """lpcnet_synthesize without a model: silence plus last_error (the
    reference would use its compiled-in model; this library has none);
    lpcnet_init on a live handle resets it (lpcnet.c:184-200 ends in
    lpcnet_reset) and keeps the model."""
    import ctypes as C
    G = np.load(os.path.join(GOLD, "streams_int8.npz"))
    net = L.LPCNet()
    out = net.synthesize(G["features"][0, 3])
    assert np.all(out == 0) and "no model" in L.last_error()
    net.load_model(blobs["streams_int8"])
    for fr in range(4):
        assert np.array_equal(net.synthesize(G["features"][0, fr]), G["pcm"][0, fr])
    assert L.lib.lpcnet_init(C.c_void_p(net._st)) == 0
    for fr in range(4):
        assert np.array_equal(net.synthesize(G["features"][0, fr]), G["pcm"][0, fr]), fr


def test_bench_preheat_computes_the_same_frames(require_gpu, blobs):
    """bench.py's preheat (untimed load for the clock ramp, then a reset of
    every stream) leaves the warmup and timed frames exactly as without it."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    blob = blobs["streams_int8"]
    _, _, _, cold = bench.run_batch(L, blob, 64, 0, 3, 6, None, 1, 0.0)
    _, _, _, warm = bench.run_batch(L, blob, 64, 0, 3, 6, None, 1, 20.0)
    assert np.array_equal(cold, warm)
    assert np.abs(cold[3:].astype(np.int64)).sum() > 0


@pytest.mark.parametrize("variant,skewed,B", [(0, False, 300), (0, False, 1030), (0, True, 1030), (0, False, 2100),
                                              (1, False, 200)])
def test_live_single_frame_chunked_matches_oracle(require_gpu, monkeypatch, variant, skewed, B):
    """The per-frame host-I/O path of large batches (lpcnet_batch_synthesize
    once per frame: a live server's 10 ms tick) runs lpc_kernel +
    chunk_kernel<1, SC> (stream-only columns) + the sample kernel reading
    the frame's outputs from FrameCond: PCM identical to the per-frame
    frame_kernel path (LPCNET_NO_CHUNK=1) on every stream and to the oracle
    on sampled streams -- through the silent FEATURES_DELAY frames, mf_kernel
    (incl. its split form for the skewed model), mf2_kernel (2100 streams,
    one ragged workgroup) and fp_kernel."""
    blob = L.synthetic_model(1, variant, skewed=skewed)
    F = 6
    allf = np.stack([feats(s, F) for s in range(B)], 1)
    b = L.LPCNetBatch(B, 0, blob)
    got = np.stack([b.synthesize(allf[f]) for f in range(F)], 1)
    b.close()
    monkeypatch.setenv("LPCNET_NO_CHUNK", "1")
    b2 = L.LPCNetBatch(B, 0, blob)
    per = np.stack([b2.synthesize(allf[f]) for f in range(F)], 1)
    b2.close()
    assert np.array_equal(got, per)
    for s in sorted({0, 1, B // 2, B - 1}):
        o = O.Oracle(blob, variant)
        assert np.array_equal(got[s], np.stack([o.synthesize(allf[f, s]) for f in range(F)])), s


@pytest.mark.parametrize("groups,B,F", [(3, 12, 5), (3, 3073, 4), (3, 4096, 6), (2, 8, 5), (2, 2049, 4),
                                        (2, 4096, 6)])
def test_wide_kernel_matches_oracle(require_gpu, monkeypatch, groups, B, F):
    """mfw_kernel (two or three 4-stream groups per workgroup, dedicated
    gather / recurrent / sampler waves): every stream equals mf2_kernel's
    (LPCNET_MFW=0) and sampled streams equal the oracle -- one workgroup (12
    or 8 streams, forced with LPCNET_MFW=1), a ragged last workgroup (3073,
    2049), multi-frame launches through the device-resident path (4096) and
    the host-I/O path (all)."""
    blob = L.synthetic_model(1, 0)
    allf = np.stack([feats(s, F) for s in range(B)], 1)
    monkeypatch.setenv("LPCNET_MF2", "1")
    monkeypatch.setenv("LPCNET_MFW", "1")
    monkeypatch.setenv("LPCNET_MFW_G", str(groups))
    b = L.LPCNetBatch(B, 0, blob)
    assert b.info().quad_path == 7 and b.info().kernel_name == f"mfw_kernel<true, {groups}, false>"
    got = np.stack([b.synthesize(allf[f]) for f in range(F)], 1)
    b.reset()
    d_f = b.device_alloc(allf.nbytes)
    d_p = b.device_alloc(F * B * 160 * 2)
    b.h2d(d_f, np.ascontiguousarray(allf))
    b.synthesize_frames(None, d_f, d_p, F)
    b.sync()
    dev = np.zeros((F, B, 160), np.int16)
    b.d2h(dev, d_p)
    b.device_free(d_f)
    b.device_free(d_p)
    b.close()
    assert np.array_equal(dev.transpose(1, 0, 2), got)
    monkeypatch.setenv("LPCNET_MFW", "0")
    b2 = L.LPCNetBatch(B, 0, blob)
    assert b2.info().quad_path in (4, 6)
    ref = np.stack([b2.synthesize(allf[f]) for f in range(F)], 1)
    b2.close()
    assert np.array_equal(got, ref)
    for s in sorted(x for x in {0, 5, 11, B // 2, B - 1} if x < B):
        o = O.Oracle(blob, 0)
        assert np.array_equal(got[s], np.stack([o.synthesize(allf[f, s]) for f in range(F)])), s


@pytest.mark.parametrize("variant,B,n,mfw", [(0, 1024, 160, "0"), (0, 1024, 80, "0"), (0, 2100, 160, "0"),
                                             (0, 3073, 160, "1"), (1, 200, 160, "0"), (0, 64, 160, "0"),
                                             (0, 4100, 160, "0")])
def test_live_engine_buffers_match_caller_buffers(require_gpu, monkeypatch, variant, B, n, mfw):
    """lpcnet_batch_synthesize on the batch's own pinned buffers
    (lpcnet_batch_host_features / _pcm): the sample kernel stores the PCM into
    the mapped host buffer itself (mf_kernel at 1024 streams, mfw_kernel at
    3073, fp_kernel at 200; N = 80 packs [B][80]), mf2_kernel (2100, 4100)
    and the small-batch path (64) go through device memory and one copy; up
    to 4096 streams the LPC and chunk kernels read the features from the
    mapped buffer -- PCM identical to the caller-buffer path with DMA-copied
    features on every stream and frame, and to the oracle on sampled
    streams."""
    monkeypatch.setenv("LPCNET_MFW", mfw)
    blob = L.synthetic_model(1, variant)
    F = 5
    allf = np.stack([feats(s, F) for s in range(B)], 1)
    b = L.LPCNetBatch(B, 0, blob)
    hf = b.host_features()
    assert hf.shape == (B, 20)
    got = []
    for f in range(F):
        np.copyto(hf, allf[f])
        got.append(np.array(b.synthesize_host(n)))
    got = np.stack(got, 1)
    b.close()
    # the caller-buffer path with the features in one DMA copy and a blocking
    # wait (the zero-copy feature reads and the polled tick end off)
    monkeypatch.setenv("LPCNET_FEAT_DMA", "1")
    monkeypatch.setenv("LPCNET_SYNC_BLOCK", "1")
    b2 = L.LPCNetBatch(B, 0, blob)
    ref = np.stack([b2.synthesize(allf[f], n) for f in range(F)], 1)
    b2.close()
    assert got.shape == (B, F, n)
    assert np.array_equal(got, ref)
    if n == 160:
        for s in sorted({0, B // 2, B - 1}):
            o = O.Oracle(blob, variant)
            assert np.array_equal(got[s], np.stack([o.synthesize(allf[f, s]) for f in range(F)])), s


def test_host_views_outlive_close(require_gpu):
    """arrays handed out by host_features() / synthesize_host()
    keep the batch's pinned memory alive past close() (no use-after-free):
    the last PCM view still reads what the frame wrote, the feature view
    stays writable, and the batch is destroyed once they go."""
    import gc
    import weakref
    blob = L.synthetic_model(1, 0)
    B = 64
    b = L.LPCNetBatch(B, 0, blob)
    hf = b.host_features()
    np.copyto(hf, np.stack([feats(s, 1)[0] for s in range(B)]))
    pcm = b.synthesize_host()
    want = np.array(pcm)
    owner = weakref.ref(b._owner)
    b.close()
    gc.collect()
    assert owner() is not None  # the views hold the native batch
    assert np.array_equal(pcm, want)
    hf[:] = 0.0
    del pcm, hf
    gc.collect()
    assert owner() is None  # destroyed with the last view


@pytest.mark.parametrize("B,F", [(8, 3), (2049, 3), (4100, 4), (8192, 2)])
def test_wide_kernel_split_form_matches_oracle(require_gpu, monkeypatch, B, F):
    """Trained-like (Sparsify, skewed) masks on the wide kernel: mfw_kernel's
    split form (block rows beyond the register caps in pieces on two host
    waves, their int32 partial sums merged through LDS adds) -- every stream
    equals mf2_kernel's split form (LPCNET_NO_MFW_SPLIT=1), host-I/O and
    device-resident multi-frame launches agree, sampled streams equal the
    oracle; one workgroup (forced), ragged (2049, 4100) and 8192 streams."""
    blob = L.synthetic_model(1, 0, skewed=True)
    allf = np.stack([feats(s, F) for s in range(B)], 1)
    if B < 1024:
        monkeypatch.setenv("LPCNET_MF2", "1")
        monkeypatch.setenv("LPCNET_MFW", "1")
    b = L.LPCNetBatch(B, 0, blob)
    info = b.info()
    assert info.quad_path == 7 and info.long_rows == 1 and info.kernel_name == "mfw_kernel<true, 2, true>"
    got = np.stack([b.synthesize(allf[f]) for f in range(F)], 1)
    b.reset()
    d_f = b.device_alloc(allf.nbytes)
    d_p = b.device_alloc(F * B * 160 * 2)
    b.h2d(d_f, np.ascontiguousarray(allf))
    b.synthesize_frames(None, d_f, d_p, F)
    b.sync()
    dev = np.zeros((F, B, 160), np.int16)
    b.d2h(dev, d_p)
    b.device_free(d_f)
    b.device_free(d_p)
    st = b.get_state(B - 1)
    b.close()
    assert np.array_equal(dev.transpose(1, 0, 2), got)
    monkeypatch.setenv("LPCNET_NO_MFW_SPLIT", "1")
    b2 = L.LPCNetBatch(B, 0, blob)
    assert b2.info().quad_path in (4, 6)
    ref = np.stack([b2.synthesize(allf[f]) for f in range(F)], 1)
    b2.reset()
    for f in range(F):
        b2.synthesize(allf[f])
    st2 = b2.get_state(B - 1)
    b2.close()
    assert np.array_equal(got, ref)
    assert np.array_equal(st["gru_a_state"].view(np.uint32), st2["gru_a_state"].view(np.uint32))
    for s in sorted(x for x in {0, 5, B // 2, B - 1} if x < B):
        o = O.Oracle(blob, 0)
        assert np.array_equal(got[s], np.stack([o.synthesize(allf[f, s]) for f in range(F)])), s
