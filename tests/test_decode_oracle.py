"""CPU checks of the 1.6 kb/s decoder restatement (oracle/lpcnet_oracle.c
oracle_decode_packet, restating /root/reference/src/lpcnet_dec.c:52-156 and
common.c:36-65) and of the reference-internal entry points the PLC drives
(lpcnet.c:122-144, 226-271).

PARITY UNPINNED by a reference build: lpcnet_dec.c and common.c include
lpcnet_private.h -> the generated nnet_data.h (absent, network-fetched), and
the codebooks are generated data (ceps_codebooks.c, absent).  The decoder is
pinned here against a second, independent numpy restatement of the same
lines (bit reader, field layout, float32 expression order), and the GPU tests
compare the device decoder with the oracle bit for bit."""
import math

import numpy as np
import pytest

import lpcnet_amd as L
import oracle_lib as O

BLOB = L.synthetic_model(1, L.VARIANT_INT8, codebooks=True)
f32 = np.float32


def codebooks(blob: bytes):
    off, out = 0, {}
    while off < len(blob):
        size, block = np.frombuffer(blob[off + 12:off + 20], np.int32)
        name = blob[off + 20:off + 64].split(b"\0")[0].decode()
        if name.startswith("ceps_codebook"):
            out[name] = np.frombuffer(blob[off + 64:off + 64 + int(size)], np.float32)
        off += 64 + int(block)
    return out


def np_decode_packet(cb, vq_mem, buf):
    """numpy float32 restatement of decode_packet (lpcnet_dec.c:81-156)."""
    bits = "".join(format(b, "08b") for b in buf)  # bits_unpack: MSB first (:52-72)
    pos = [0]

    def take(n):
        v = int(bits[pos[0]:pos[0] + n], 2)
        pos[0] += n
        return v
    c0_id, main_pitch, modulation, corr_id = take(7), take(6), take(3), take(2)
    vq_end = [take(10), take(10), take(10)]
    vq_mid, interp_id = take(13), take(3)
    F = np.zeros((4, 36), np.float32)
    modulation -= 4
    voiced = modulation != -4
    if not voiced:
        modulation = 0
    frame_corr = f32(0.3875) + f32(0.175) * f32(corr_id) if voiced else f32(0.0375) + f32(0.075) * f32(corr_id)
    for sub in range(4):
        p = f32(math.pow(2.0, main_pitch / 21.0) * 32)
        p = f32(p * (f32(1) + f32(f32(f32(modulation) / f32(16)) / f32(7)) * f32(2 * sub - 3)))
        p = min(f32(255), max(f32(33), p))
        F[sub, 18] = f32(0.02) * (p - f32(100))
        F[sub, 19] = frame_corr - f32(0.5)
    F[3, 0] = f32(c0_id - 64) / f32(4)
    c1, c2, c3, cd = (cb["ceps_codebook1"].reshape(1024, 17), cb["ceps_codebook2"].reshape(1024, 17),
                      cb["ceps_codebook3"].reshape(1024, 17), cb["ceps_codebook_diff4"].reshape(4096, 18))
    F[3, 1:18] = (c1[vq_end[0]] + c2[vq_end[1]]) + c3[vq_end[2]]
    sign = f32(1)
    if vq_mid >= 4096:
        vq_mid -= 4096
        sign = f32(-1)
    F[1, :18] = sign * cd[vq_mid]
    if (vq_mid & 3) < 2:
        F[1, :18] += f32(0.5) * (vq_mem + F[3, :18])
    elif (vq_mid & 3) == 2:
        F[1, :18] += vq_mem
    else:
        F[1, :18] += F[3, :18]
    best = interp_id + (interp_id >= 7)
    preds = lambda l, r: [f32(0.5) * (l + r), l, r]  # noqa: E731  common.c:36-56
    F[0, :18] = preds(vq_mem, F[1, :18])[best // 3]
    F[2, :18] = preds(F[1, :18], F[3, :18])[best % 3]
    return F, F[3, :18].copy()


def random_packets(n, seed=7):
    return np.random.default_rng(seed).integers(0, 256, size=(n, 8), dtype=np.uint8)


def test_oracle_decode_packet_matches_numpy_restatement():
    cb = codebooks(BLOB)
    assert set(cb) == {"ceps_codebook1", "ceps_codebook2", "ceps_codebook3", "ceps_codebook_diff4"}
    o = O.Oracle(BLOB)
    mem = np.zeros(18, np.float32)
    pk = random_packets(400)
    # every interp id, every vq_mid class, unvoiced and voiced, both signs
    pk[:8, 7] = (pk[:8, 7] & 0xF8) | np.arange(8)
    pk[8:12, 1] &= 0xF8  # modulation bits 13..15 -> 0 = unvoiced for a few
    for buf in pk:
        got = o.decode_packet(bytes(buf))
        want, mem = np_decode_packet(cb, mem, bytes(buf))
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), buf


def test_oracle_decode_needs_codebooks():
    o = O.Oracle(L.synthetic_model(1, L.VARIANT_INT8))
    with pytest.raises(ValueError):
        o.decode_packet(bytes(8))


def test_codebook_records_do_not_change_synthesis_arrays():
    base = L.synthetic_model(1, L.VARIANT_INT8)
    assert BLOB[:len(base)] == base
    L.validate_model(BLOB)
    feats = L.synthetic_features(0, 6)
    assert np.array_equal(O.synth_stream(BLOB, feats[:, :20]), O.synth_stream(base, feats[:, :20]))


def test_oracle_flush_keeps_conditioning():
    """run_frame_network_flush writes the frame network's outputs into locals
    (lpcnet.c:134-144): conditioning and LPC stay, frame_count advances."""
    o = O.Oracle(L.synthetic_model(1, L.VARIANT_INT8))
    feats = L.synthetic_features(3, 8)
    for f in range(4):
        o.synthesize(feats[f])
    a0, b0, l0 = o.frame()
    fc0 = o.frame_count()
    o.frame_deferred(feats[4])
    o.frame_deferred(feats[5])
    o.frame_flush()
    a1, b1, l1 = o.frame()
    assert o.frame_count() == fc0 + 2
    assert np.array_equal(a0, a1) and np.array_equal(b0, b1) and np.array_equal(l0, l1)
    # deferred keeps the last 4 (lpcnet.c:122-132): 6 deferred frames flush 4
    for f in range(6):
        o.frame_deferred(feats[f % 8])
    o.frame_flush()
    assert o.frame_count() == fc0 + 6


def test_oracle_snapshot_round_trip():
    o = O.Oracle(L.synthetic_model(1, L.VARIANT_INT8))
    feats = L.synthetic_features(5, 6)
    for f in range(3):
        o.synthesize(feats[f])
    snap = o.save()
    a = [o.synthesize(feats[f]) for f in range(3, 6)]
    o.restore(snap)
    b = [o.synthesize(feats[f]) for f in range(3, 6)]
    assert np.array_equal(np.stack(a), np.stack(b))


def test_append_codebooks_tool_round_trip(tmp_path):
    """tools/append_codebooks.py rebuilds the codebook-carrying blob from a
    plain blob and the concatenated codebook arrays; appending again replaces
    the records instead of duplicating them."""
    import subprocess
    import sys
    import os
    cb = codebooks(BLOB)
    flat = np.concatenate([cb["ceps_codebook1"], cb["ceps_codebook2"], cb["ceps_codebook3"],
                           cb["ceps_codebook_diff4"]]).astype("<f4")
    base = L.synthetic_model(1, L.VARIANT_INT8)
    (tmp_path / "w.bin").write_bytes(base)
    flat.tofile(tmp_path / "cb.f32")
    tool = os.path.join(O.ROOT, "tools", "append_codebooks.py")
    for src in ("w.bin", "out.bin"):
        subprocess.run([sys.executable, tool, str(tmp_path / src), str(tmp_path / "cb.f32"), str(tmp_path / "out.bin")],
                       check=True)
        assert (tmp_path / "out.bin").read_bytes() == BLOB
    bad = subprocess.run([sys.executable, tool, str(tmp_path / "w.bin"), str(tmp_path / "w.bin"),
                          str(tmp_path / "x.bin")], capture_output=True)
    assert bad.returncode != 0
