"""Host-side checks that need no GPU: the C-ABI library loads and exports every
symbol declared in include/*.h, the rcpps table, and the synthetic
generator's determinism."""
import hashlib
import os
import re

import numpy as np
import pytest

import lpcnet_amd as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K = np.load(os.path.join(ROOT, "tests", "golden", "kernels.npz"))


def declared_symbols():
    syms = []
    for h in ("lpcnet.h", "lpcnet_mi355x.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        syms += re.findall(r"^LPCNET_EXPORT[^;(]*?\b(\w+)\s*\(", txt, re.M)
    return syms


def test_library_exports_every_declared_symbol():
    syms = declared_symbols()
    assert len(syms) >= 30
    for s in syms:
        assert hasattr(L.lib, s), s


def test_reference_api_subset_present():
    for s in ("lpcnet_get_size", "lpcnet_init", "lpcnet_create", "lpcnet_destroy", "lpcnet_reset",
              "lpcnet_synthesize", "lpcnet_load_model"):
        assert s in declared_symbols()


def test_rcp_table_matches_fixture():
    tab = np.fromfile(os.path.join(ROOT, "tests", "golden", "rcp_x86.bin"), np.uint32)
    assert np.array_equal(L.rcp_table(), tab)


def test_synthetic_model_deterministic_and_layout():
    a = L.synthetic_model(1, L.VARIANT_INT8)
    b = L.synthetic_model(1, L.VARIANT_INT8)
    c = L.synthetic_model(2, L.VARIANT_INT8)
    assert a == b and a != c
    G = np.load(os.path.join(ROOT, "tests", "golden", "streams_int8.npz"))
    assert hashlib.sha256(a).digest() == G["blob_sha256"].tobytes()
    # every record: 64-byte WeightHead, 64-aligned payload (nnet.h:54-61)
    off, names = 0, []
    while off < len(a):
        assert a[off:off + 4] == b"DNNw"
        size, block = np.frombuffer(a[off + 12:off + 20], np.int32)
        assert block % 64 == 0 and block >= size
        names.append(a[off + 20:off + 64].split(b"\0")[0].decode())
        off += 64 + int(block)
    assert off == len(a)
    assert "sparse_gru_a_recurrent_weights_idx" in names and "dual_fc_factor" in names


def test_synthetic_features_shape():
    f = L.synthetic_features(3, 5)
    assert f.shape == (5, 36) and np.all(f[:, 20:] == 0)
    assert np.all((f[:, 18] >= -1.3) & (f[:, 18] <= 1.5))


def test_batch_create_fails_cleanly_without_device():
    if L.device_count() > 0:
        return
    import pytest
    with pytest.raises(L.LPCNetError):
        L.LPCNetBatch(4)


def test_kernel_float_identities_exhaustive(tmp_path):
    """The HIP kernels replace lin2ulaw's float division and the
    floor(.5 + (double)x) roundings with exact float forms; this proves them
    over every float input they can see (oracle/checks/exact_identities.c)."""
    import subprocess
    exe = tmp_path / "exact_identities"
    src = os.path.join(ROOT, "oracle", "checks", "exact_identities.c")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), src, "-lm"], check=True)
    r = subprocess.run([str(exe), os.path.join(ROOT, "tests", "golden", "rcp_x86.bin")], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout


def test_lpcnet_init_never_trusts_raw_memory():
    """lpcnet_init runs on caller memory (lpcnet_get_size + malloc, as the
    reference's decoder does): bytes that look like a live handle (the magic
    word and a stray batch pointer, e.g. a block a scrub-free allocator
    reused after lpcnet_destroy) must give a fresh handle, never a reset of
    that pointer.  Re-init of a live handle and destroy stay well-defined.
    No device work: the batch is bound lazily by lpcnet_load_model."""
    import ctypes as C
    n = L.lib.lpcnet_get_size()
    raw = (C.c_ubyte * n)()
    C.memmove(raw, (0x4c50434e).to_bytes(4, "little") + b"\0" * 4 + (0xdeadbeef000).to_bytes(8, "little"), 16)
    assert L.lib.lpcnet_init(C.cast(raw, C.c_void_p)) == 0
    assert L.lib.lpcnet_init(C.cast(raw, C.c_void_p)) == 0  # now live: re-init resets (nothing bound)
    st = L.lib.lpcnet_create()
    assert st
    L.lib.lpcnet_destroy(st)
    st2 = L.lib.lpcnet_create()  # may reuse the freed block
    assert st2 and L.lib.lpcnet_init(st2) == 0
    L.lib.lpcnet_destroy(st2)


def test_device_numerics_rejects_bad_arguments():
    """Argument checks happen before any HIP call (no GPU needed)."""
    assert L.lib.lpcnet_mi355x_device_numerics(0, 99, None, None, 1) == -1
    assert L.lib.lpcnet_mi355x_device_numerics(0, 0, None, None, 4) == -1
    assert L.lib.lpcnet_mi355x_device_numerics(0, 0, None, None, 0) == 0


def test_stale_registry_entry_is_dropped():
    """An LPCNetState embedded in caller memory that is freed without
    lpcnet_destroy leaves a registry entry; memory reused at that address
    (garbage, or another handle's bytes) must start a fresh handle -- the
    registry's record, never the memory, says what to release."""
    import ctypes as C
    n = L.lib.lpcnet_get_size()
    raw = (C.c_ubyte * n)()
    p = C.cast(raw, C.c_void_p)
    assert L.lib.lpcnet_init(p) == 0
    snap = bytes(raw)
    C.memmove(raw, b"\x5a" * n, n)  # the block reused for something else
    assert L.lib.lpcnet_init(p) == 0  # stale entry dropped, fresh handle
    assert bytes(raw) != snap  # a new token
    C.memmove(raw, snap, n)  # the old handle's bytes: not the live token any more
    assert L.lib.lpcnet_init(p) == 0
    L.lib.lpcnet_mi355x_deinit(p)
    assert bytes(raw[:4]) == b"\0\0\0\0"
    L.lib.lpcnet_mi355x_deinit(p)  # idempotent
    # an embedded decoder state: init / destroy without a device
    d = L.lib.lpcnet_decoder_create()
    assert d and L.lib.lpcnet_decoder_init(d) == 0
    L.lib.lpcnet_decoder_destroy(d)


def test_handle_entry_points_fail_cleanly_without_model():
    """The reference-internal entry points on a handle with no model bound:
    silence out, no crash, no device work."""
    import ctypes as C
    st = L.lib.lpcnet_create()
    out = np.full(160, 7, np.int16)
    f = np.zeros(20, np.float32)
    L.lib.lpcnet_synthesize_impl(st, f.ctypes.data, out.ctypes.data, 160, 10)
    assert np.all(out == 0)
    out[:] = 7
    L.lib.lpcnet_synthesize_tail_impl(st, out.ctypes.data, 160, 0)
    assert np.all(out == 0)
    L.lib.run_frame_network_deferred(st, f.ctypes.data)
    L.lib.run_frame_network_flush(st)
    L.lib.lpcnet_reset_signal(st)
    buf = C.create_string_buffer(L.lib.lpcnet_mi355x_state_size())
    assert L.lib.lpcnet_mi355x_state_save(st, buf) == -1
    d = L.lib.lpcnet_decoder_create()
    pcm = np.full(640, 3, np.int16)
    assert L.lib.lpcnet_decode(d, bytes(8), pcm.ctypes.data) == -1 and np.all(pcm == 0)
    L.lib.lpcnet_decoder_destroy(d)
    L.lib.lpcnet_destroy(st)


def test_placement_policy_without_gpu():
    """Drop-in placement (no device touched before a model is bound): handles
    go to the least-loaded placement of the list (counted from the last
    lpcnet_mi355x_set_placement on; earlier handles keep theirs); a device
    index outside the visible ones is refused; LPCNET_DEVICE pins
    (placement -1)."""
    import gc
    import os
    gc.collect()
    L.set_placement([0, 0, 0])
    try:
        nets = [L.LPCNet() for _ in range(7)]
        assert [n.placement() for n in nets] == [(0, k % 3) for k in range(7)]
        with pytest.raises(L.LPCNetError):
            L.set_placement([-1])
        nets[1].close()
        nets[4].close()
        late = L.LPCNet()  # placement 1 had 2 live handles, now none
        assert late.placement() == (0, 1)
        os.environ["LPCNET_DEVICE"] = "0"
        try:
            pinned = L.LPCNet()
            assert pinned.placement() == (0, -1)
        finally:
            del os.environ["LPCNET_DEVICE"]
        for n in nets + [late, pinned]:
            n.close()
    finally:
        gc.collect()
        L.set_placement([])


INIT_NO_HIP = r"""
import os, sys
sys.path.insert(0, sys.argv[1])
os.environ.pop("LOCAL_RANK", None)
os.environ.pop("LPCNET_DEVICES", None)
import lpcnet_amd as L


def kfd_open():
    fds = os.listdir("/proc/self/fd")
    out = []
    for fd in fds:
        try:
            out.append(os.readlink("/proc/self/fd/" + fd))
        except OSError:
            pass
    return any(p.startswith("/dev/kfd") or p.startswith("/dev/dri") for p in out)


nets = [L.LPCNet() for _ in range(4)]
assert [n.placement() for n in nets] == [(0, 0)] * 4, [n.placement() for n in nets]
assert not kfd_open(), "lpcnet_init / lpcnet_create started the HIP runtime"
for n in nets:
    n.close()
print("ok")
"""


def test_init_leaves_hip_uninitialised():
    """lpcnet_init / lpcnet_create with the default placement
    must not start the HIP runtime (a caller may fork workers or exec after
    creating handles, before binding a model): a fresh process creates
    handles, queries their placement (one placement, device 0 without
    LOCAL_RANK) and has not opened /dev/kfd."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, "-c", INIT_NO_HIP, ROOT], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr


def test_bad_device_list_fails_init():
    """LPCNET_DEVICES is checked when the first handle is placed: a malformed
    list makes lpcnet_init fail (lpcnet_create returns NULL) instead of being
    ignored."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, sys.argv[1]); import lpcnet_amd as L\n"
            "assert not L.lib.lpcnet_create()\n"
            "assert 'LPCNET_DEVICES' in L.last_error(), L.last_error()\nprint('ok')")
    env = dict(os.environ, LPCNET_DEVICES="0,x")
    r = subprocess.run([sys.executable, "-c", code, ROOT], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr


def test_bench_line_serialises_numpy_scalars():
    """the bench line's ladders hold numpy-derived values (np.bool_ realtime
    flags, np.float64 means): the line must still print as JSON"""
    import json
    import sys
    sys.path.insert(0, ROOT)
    import bench
    row = {"realtime": np.float64(3.0) <= 10.0, "ms": np.float64(3.0), "n": np.int64(4)}
    assert json.loads(json.dumps(row, default=bench._json_scalar)) == {"realtime": True, "ms": 3.0, "n": 4}
    with pytest.raises(TypeError):
        json.dumps({"x": object()}, default=bench._json_scalar)


def test_owned_view_keeps_owner_alive():
    """lpcnet_amd._owned_view: the array (and any slice of it) holds its
    owner; the owner's release runs only when the last view is gone."""
    import ctypes as C
    import gc
    released = []

    class Owner(L._BatchOwner):
        def __del__(self):
            released.append(True)

    mem = (C.c_int16 * 64)()
    o = Owner(None)
    v = L._owned_view(o, C.addressof(mem), C.c_int16, np.int16, (4, 16))
    del o
    gc.collect()
    s = v[1:3]
    del v
    gc.collect()
    assert not released
    s[:] = 5
    assert mem[16] == 5
    del s
    gc.collect()
    assert released == [True]


def test_wide_split_plan_host_only():
    """lpcnet_mi355x_wide_plan (host only): the default synthetic model needs
    no split; the trained-like skewed one (Sparsify masks, block rows up to
    76 / 59 / 96 blocks) gets the wide kernel's split form -- R waves within
    the register caps (<= 4 z/r and 8 h slot groups), its pieces (one per
    host lane group and gate, <= 16 per gate) on the two host waves."""
    import ctypes as C
    f = L.lib.lpcnet_mi355x_wide_plan
    f.restype = C.c_int
    out = (C.c_int * 24)()
    blob = L.synthetic_model(1, 0)
    assert f(blob, len(blob), out) == 0 and out[0] == 0 and out[1] == 0
    blob = L.synthetic_model(1, 0, skewed=True)
    assert f(blob, len(blob), out) == 0 and out[0] == 1 and out[1] == 1
    groups = [(out[2 + 2 * w], out[3 + 2 * w]) for w in range(8)]
    assert all(1 <= z <= 4 and 1 <= h <= 8 for z, h in groups), groups
    assert all(0 < n <= 16 for n in out[18:21]), list(out[18:21])
