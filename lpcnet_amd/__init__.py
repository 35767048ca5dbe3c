"""lpcnet_amd -- Python mirror of the MI355X LPCNet synthesis engine.

Thin ctypes binding over ``liblpcnet_mi355x.so`` (built in-tree by
``make lib``).  The class API mirrors the reference C interface of
``include/lpcnet.h`` (auliaadila/LPCNet):

* :class:`LPCNet` -- one stream: ``lpcnet_create`` / ``lpcnet_load_model`` /
  ``lpcnet_synthesize`` / ``lpcnet_reset`` / ``lpcnet_destroy``
  (reference ``src/lpcnet.c:174-281``).
* :class:`LPCNetBatch` -- B independent streams on one GPU (the batch extension
  of ``include/lpcnet_mi355x.h``).

There is no CPU fallback: every synthesis call runs the HIP kernels, and
importing the package raises if the native library is absent.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# LPCNET_LIB_VARIANT=<name> loads liblpcnet_mi355x_<name>.so from this
# directory instead (in-tree A/B builds; still the native library, never a fallback)
LIB_PATH = os.path.join(_HERE, "liblpcnet_mi355x%s.so" % (
    "_" + os.environ["LPCNET_LIB_VARIANT"] if os.environ.get("LPCNET_LIB_VARIANT") else ""))

NB_FEATURES = 20
NB_TOTAL_FEATURES = 36
FRAME_SIZE = 160
VARIANT_INT8 = 0
VARIANT_FP32 = 1


class LPCNetError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} not found: build it with `make lib` (or __graft_entry__.build()); "
            "lpcnet_amd has no CPU fallback")
    lib = C.CDLL(LIB_PATH)
    vp, i, f, u = C.c_void_p, C.c_int, C.c_float, C.c_uint
    sig = {
        "lpcnet_get_size": (i, []),
        "lpcnet_init": (i, [vp]),
        "lpcnet_create": (vp, []),
        "lpcnet_destroy": (None, [vp]),
        "lpcnet_reset": (None, [vp]),
        "lpcnet_synthesize": (None, [vp, vp, vp, i]),
        "lpcnet_load_model": (i, [vp, C.c_char_p, i]),
        "lpcnet_batch_create": (vp, [i, i]),
        "lpcnet_batch_destroy": (None, [vp]),
        "lpcnet_batch_load_model": (i, [vp, C.c_char_p, i]),
        "lpcnet_batch_model_info": (i, [vp, vp]),
        "lpcnet_batch_set_kernel": (i, [vp, i]),
        "lpcnet_batch_set_model_constants": (i, [vp, f, i, i]),
        "lpcnet_batch_set_rcp_table": (i, [vp, vp]),
        "lpcnet_mi355x_host_rcp_table": (i, [vp, i]),
        "lpcnet_mi355x_pool_stats": (i, [vp, vp, vp, vp]),
        "lpcnet_mi355x_set_placement": (i, [vp, i]),
        "lpcnet_mi355x_handle_placement": (i, [vp, vp, vp]),
        "lpcnet_batch_reset": (None, [vp]),
        "lpcnet_batch_reset_stream": (i, [vp, i]),
        "lpcnet_batch_nb_streams": (i, [vp]),
        "lpcnet_batch_synthesize": (i, [vp, vp, vp, i]),
        "lpcnet_batch_host_features": (C.POINTER(C.c_float), [vp]),
        "lpcnet_batch_host_pcm": (C.POINTER(C.c_short), [vp]),
        "lpcnet_batch_synthesize_impl": (i, [vp, vp, vp, i, i]),
        "lpcnet_batch_state_size": (i, []),
        "lpcnet_batch_save_state": (i, [vp, i, vp]),
        "lpcnet_batch_restore_state": (i, [vp, i, vp]),
        "lpcnet_batch_synthesize_frames": (i, [vp, vp, vp, vp, i, i]),
        "lpcnet_batch_sync": (i, [vp]),
        "lpcnet_batch_set_spin_limit": (i, [vp, i]),
        "lpcnet_batch_set_frame_chunking": (i, [vp, i]),
        "lpcnet_mi355x_validate_model": (i, [C.c_char_p, i]),
        "lpcnet_batch_device_alloc": (vp, [vp, C.c_size_t]),
        "lpcnet_batch_device_free": (i, [vp, vp]),
        "lpcnet_batch_memcpy_h2d": (i, [vp, vp, vp, C.c_size_t]),
        "lpcnet_batch_memcpy_d2h": (i, [vp, vp, vp, C.c_size_t]),
        "lpcnet_batch_reset_timers": (None, [vp, i]),
        "lpcnet_batch_kernel_ms": (C.c_double, [vp, i, C.POINTER(C.c_int)]),
        "lpcnet_batch_kernel_frames": (i, [vp, i]),
        "lpcnet_batch_set_stamps": (i, [vp, i]),
        "lpcnet_batch_get_stamps": (i, [vp, vp]),
        "lpcnet_batch_get_frame_stamps": (i, [vp, vp]),
        "lpcnet_batch_set_trace": (i, [vp, i]),
        "lpcnet_batch_get_trace": (i, [vp, vp, vp]),
        "lpcnet_batch_get_state": (i, [vp, i, vp, vp, vp, vp, vp, vp]),
        "lpcnet_mi355x_synthetic_model": (i, [u, i, i, vp, i]),
        "lpcnet_mi355x_synthetic_features": (None, [u, i, vp]),
        "lpcnet_mi355x_device_lpc": (i, [i, vp, vp, i]),
        "lpcnet_mi355x_rcp_table": (C.POINTER(C.c_uint32), []),
        "lpcnet_mi355x_device_count": (i, []),
        "lpcnet_mi355x_device_numerics": (i, [i, i, vp, vp, i]),
        "lpcnet_mi355x_last_error": (C.c_char_p, []),
        # reference-internal entry points on a handle (lpcnet_private.h:126-132)
        "lpcnet_synthesize_impl": (None, [vp, vp, vp, i, i]),
        "lpcnet_synthesize_tail_impl": (None, [vp, vp, i, i]),
        "run_frame_network_deferred": (None, [vp, vp]),
        "run_frame_network_flush": (None, [vp]),
        "lpcnet_reset_signal": (None, [vp]),
        "lpcnet_mi355x_state_size": (i, []),
        "lpcnet_mi355x_state_save": (i, [vp, vp]),
        "lpcnet_mi355x_state_restore": (i, [vp, vp]),
        "lpcnet_mi355x_deinit": (None, [vp]),
        # 1.6 kb/s decoder (include/lpcnet.h:63-100)
        "lpcnet_decoder_get_size": (i, []),
        "lpcnet_decoder_init": (i, [vp]),
        "lpcnet_decoder_create": (vp, []),
        "lpcnet_decoder_destroy": (None, [vp]),
        "lpcnet_decode": (i, [vp, vp, vp]),
        "lpcnet_mi355x_decoder_load_model": (i, [vp, C.c_char_p, i]),
        "lpcnet_batch_synthesize_tail_impl": (i, [vp, vp, i, i]),
        "lpcnet_batch_run_frame_network": (i, [vp, vp, i]),
        "lpcnet_batch_reset_signal": (i, [vp, i]),
        "lpcnet_batch_decode": (i, [vp, vp, vp]),
        "lpcnet_batch_decode_frames": (i, [vp, vp, vp, i]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


class ModelInfo(C.Structure):
    _fields_ = [("variant", C.c_int), ("gru_a_blocks", C.c_int), ("gru_b_blocks", C.c_int),
                ("may_saturate", C.c_int), ("bytes_shared_per_frame", C.c_double),
                ("bytes_shared_per_sample", C.c_double), ("bytes_per_stream_sample", C.c_double),
                ("ops_per_sample", C.c_double), ("streams_per_workgroup", C.c_int), ("quad_path", C.c_int),
                ("lds_bytes", C.c_int), ("mfma_ops_per_group_sample", C.c_double),
                ("lpc_gamma", C.c_float), ("features_delay", C.c_int), ("end2end", C.c_int),
                ("long_rows", C.c_int), ("has_codebooks", C.c_int), ("rcp_hw", C.c_int)]

    @property
    def kernel_name(self) -> str:
        """Demangled template instance of the sample kernel this model runs
        (as rocprofv3 names it)."""
        sat = "true" if self.may_saturate else "false"
        lr = "true" if self.long_rows else "false"
        hw = "true" if self.rcp_hw else "false"
        if self.quad_path == 4:
            return f"mf_kernel<{self.streams_per_workgroup}, 0, {lr}, {hw}>"
        if self.quad_path == 6:
            return f"mf2_kernel<4, {lr}, {hw}>"
        if self.quad_path == 7:
            return f"mfw_kernel<true, {self.streams_per_workgroup // 4}, {lr}>"
        if self.quad_path == 5:
            return f"fp_kernel<0, {lr}, {hw}>"
        quad = "true" if self.quad_path == 1 else "false"
        return f"sample_kernel<{self.streams_per_workgroup}, {self.variant}, {sat}, {quad}>"


def last_error() -> str:
    return (lib.lpcnet_mi355x_last_error() or b"").decode()


def device_numerics(op: int, x: np.ndarray, n: int | None = None, device: int = 0) -> np.ndarray:
    """Run one device-numerics routine (see lpcnet_mi355x_device_numerics)
    on the GPU; x is reinterpreted as 32-bit words, the result is uint32."""
    src = np.ascontiguousarray(x).view(np.uint32)
    cnt = int(n if n is not None else src.size)
    out = np.zeros(cnt, np.uint32)
    if lib.lpcnet_mi355x_device_numerics(device, op, src.ctypes.data, out.ctypes.data, cnt) != 0:
        raise LPCNetError("device numerics failed: " + last_error())
    return out


def validate_model(blob: bytes) -> None:
    """Host-only check of a weight blob with lpcnet_load_model's rules; raises LPCNetError."""
    if lib.lpcnet_mi355x_validate_model(blob, len(blob)) != 0:
        raise LPCNetError(last_error())


def device_count() -> int:
    return lib.lpcnet_mi355x_device_count()


def set_placement(devices) -> None:
    """Placement list of drop-in handles initialised from now on (a device
    may appear twice); [] restores the default (every visible device)."""
    arr = (C.c_int * max(len(devices), 1))(*devices)
    if lib.lpcnet_mi355x_set_placement(arr, len(devices)) != 0:
        raise LPCNetError(last_error())


def synthetic_model(seed: int = 1, variant: int = VARIANT_INT8, saturating: bool = False, skewed: bool = False,
                    codebooks: bool = False) -> bytes:
    """Deterministic synthetic default-size model in the reference blob format.
    skewed: GRU_A masks by a global per-gate threshold over skewed block
    energies (Sparsify, training_tf2/lpcnet.py:140-160): long block rows.
    codebooks: append the 1.6 kb/s decoder's ceps codebooks (other arrays unchanged)."""
    flags = (1 if saturating else 0) | (2 if skewed else 0) | (4 if codebooks else 0)
    n = lib.lpcnet_mi355x_synthetic_model(seed, variant, flags, None, 0)
    buf = C.create_string_buffer(n)
    lib.lpcnet_mi355x_synthetic_model(seed, variant, flags, buf, n)
    return buf.raw


def with_model_constants(blob: bytes, lpc_gamma: float | None = None, features_delay: int | None = None,
                         end2end: bool | None = None) -> bytes:
    """``blob`` plus the side records LPC_GAMMA / FEATURES_DELAY / END2END
    (64-byte WeightHead records, nnet.h:54-61) that carry the constants
    dump_lpcnet.py writes into nnet_data.h; the reference's parser skips
    records it does not bind."""
    out = bytearray(blob)
    for name, val in (("LPC_GAMMA", None if lpc_gamma is None else np.float32(lpc_gamma).tobytes()),
                      ("FEATURES_DELAY", None if features_delay is None else np.int32(features_delay).tobytes()),
                      ("END2END", None if end2end is None else np.int32(1 if end2end else 0).tobytes())):
        if val is None:
            continue
        head = bytearray(64)
        head[0:4] = b"DNNw"
        head[8:12] = np.int32(0 if name == "LPC_GAMMA" else 1).tobytes()  # WEIGHT_TYPE_float / _int
        head[12:16] = np.int32(4).tobytes()
        head[16:20] = np.int32(64).tobytes()
        head[20:20 + len(name)] = name.encode()
        out += head + val + bytes(60)
    return bytes(out)


def synthetic_features(stream: int, nframes: int) -> np.ndarray:
    """[nframes, 36] float32 synthetic features of stream ``stream``."""
    out = np.zeros((nframes, NB_TOTAL_FEATURES), np.float32)
    lib.lpcnet_mi355x_synthetic_features(stream, nframes, out.ctypes.data)
    return out


def device_lpc(cepstra: np.ndarray, device: int = 0) -> np.ndarray:
    """lpc_from_cepstrum (freq.c:310-320) of cepstra [n, 18] on the GPU (lpc_kernel) -> [n, 16]."""
    c = np.ascontiguousarray(np.asarray(cepstra, np.float32).reshape(-1, 18))
    out = np.zeros((c.shape[0], 16), np.float32)
    if lib.lpcnet_mi355x_device_lpc(device, c.ctypes.data, out.ctypes.data, c.shape[0]) != 0:
        raise LPCNetError("device LPC failed: " + last_error())
    return out


def host_rcp_table() -> tuple[np.ndarray, int]:
    """This host CPU's rcpps as the 4096-entry (top 12 mantissa bits) table
    and the number of mantissas/exponents that form does not reproduce."""
    t = np.zeros(4096, np.uint32)
    bad = lib.lpcnet_mi355x_host_rcp_table(t.ctypes.data, 4096)
    return t, bad


def rcp_table() -> np.ndarray:
    p = lib.lpcnet_mi355x_rcp_table()
    return np.ctypeslib.as_array(p, shape=(2048,)).copy()


class LPCNet:
    """One synthesis stream (reference LPCNetState semantics)."""

    def __init__(self, blob: bytes | None = None):
        self._st = lib.lpcnet_create()
        if not self._st:
            raise LPCNetError("lpcnet_create failed")
        if blob is not None:
            self.load_model(blob)

    def load_model(self, blob: bytes) -> None:
        if lib.lpcnet_load_model(self._st, blob, len(blob)) != 0:
            raise LPCNetError(f"lpcnet_load_model failed: {last_error()}")

    def reset(self) -> None:
        lib.lpcnet_reset(self._st)

    def synthesize(self, features: np.ndarray, n: int = FRAME_SIZE) -> np.ndarray:
        f = np.ascontiguousarray(features[:NB_FEATURES], np.float32)
        out = np.zeros(n, np.int16)
        lib.lpcnet_synthesize(self._st, f.ctypes.data, out.ctypes.data, n)
        return out

    # -- reference-internal entry points (lpcnet_private.h:126-132, the PLC's calls) --
    def synthesize_impl(self, features: np.ndarray, pcm: np.ndarray, preload: int) -> np.ndarray:
        """lpcnet_synthesize_impl: pcm [N] int16, the first ``preload`` samples teacher-forced."""
        f = np.ascontiguousarray(np.asarray(features, np.float32)[:NB_FEATURES])
        out = np.ascontiguousarray(pcm, np.int16).copy()
        lib.lpcnet_synthesize_impl(self._st, f.ctypes.data, out.ctypes.data if out.size else None, out.size, preload)
        return out

    def synthesize_tail_impl(self, pcm: np.ndarray, preload: int = 0) -> np.ndarray:
        """lpcnet_synthesize_tail_impl: the sample network only, on the current conditioning."""
        out = np.ascontiguousarray(pcm, np.int16).copy()
        lib.lpcnet_synthesize_tail_impl(self._st, out.ctypes.data if out.size else None, out.size, preload)
        return out

    def frame_deferred(self, features: np.ndarray) -> None:
        """run_frame_network_deferred (lpcnet.c:122-132)."""
        f = np.ascontiguousarray(np.asarray(features, np.float32)[:NB_FEATURES])
        lib.run_frame_network_deferred(self._st, f.ctypes.data)

    def frame_flush(self) -> None:
        """run_frame_network_flush (lpcnet.c:134-144)."""
        lib.run_frame_network_flush(self._st)

    def reset_signal(self) -> None:
        """lpcnet_reset_signal (lpcnet.c:226-233)."""
        lib.lpcnet_reset_signal(self._st)

    def save(self) -> bytes:
        """The handle's whole synthesis state (replaces the PLC's LPCNetState struct copy)."""
        buf = C.create_string_buffer(lib.lpcnet_mi355x_state_size())
        if lib.lpcnet_mi355x_state_save(self._st, buf) != 0:
            raise LPCNetError(last_error())
        return buf.raw

    def restore(self, state: bytes) -> None:
        if lib.lpcnet_mi355x_state_restore(self._st, state) != 0:
            raise LPCNetError(last_error())

    def placement(self) -> tuple[int, int]:
        """(device, placement index; -1 when pinned by LPCNET_DEVICE)."""
        d, p = C.c_int(), C.c_int()
        if lib.lpcnet_mi355x_handle_placement(self._st, C.byref(d), C.byref(p)) != 0:
            raise LPCNetError(last_error())
        return d.value, p.value

    def close(self) -> None:
        if self._st:
            lib.lpcnet_destroy(self._st)
            self._st = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class LPCNetDecoder:
    """The 1.6 kb/s decoder: lpcnet_decoder_create / lpcnet_decode (lpcnet.c:283-319)."""

    def __init__(self, blob: bytes):
        self._st = lib.lpcnet_decoder_create()
        if not self._st:
            raise LPCNetError("lpcnet_decoder_create failed")
        if lib.lpcnet_mi355x_decoder_load_model(self._st, blob, len(blob)) != 0:
            err = last_error()
            self.close()
            raise LPCNetError(f"decoder model: {err}")

    def decode(self, packet: bytes) -> np.ndarray:
        """One 8-byte packet -> 640 int16 samples."""
        if len(packet) != 8:
            raise ValueError("a packet is 8 bytes")
        buf = C.create_string_buffer(bytes(packet), 8)
        out = np.zeros(4 * FRAME_SIZE, np.int16)
        if lib.lpcnet_decode(self._st, buf, out.ctypes.data) != 0:
            raise LPCNetError(last_error())
        return out

    def close(self) -> None:
        if self._st:
            lib.lpcnet_decoder_destroy(self._st)
            self._st = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _BatchOwner:
    """Owns the native batch: lpcnet_batch_destroy runs when the last
    reference goes -- the LPCNetBatch (until close()) or an array handed out
    by host_features() / synthesize_host(), whose buffer object holds this
    owner, so such an array never outlives the host-visible memory it views."""

    def __init__(self, ptr):
        self.ptr = ptr

    def __del__(self):
        if self.ptr:
            lib.lpcnet_batch_destroy(self.ptr)
            self.ptr = None


def _owned_view(owner: _BatchOwner, addr: int, ctype, dtype, shape) -> np.ndarray:
    n = int(np.prod(shape))
    buf = (ctype * n).from_address(addr)
    buf._owner = owner  # the array's base keeps the native batch alive
    return np.frombuffer(buf, dtype=dtype).reshape(shape)


class LPCNetBatch:
    """B independent streams on one MI355X (include/lpcnet_mi355x.h)."""

    def __init__(self, nb_streams: int, device: int = 0, blob: bytes | None = None):
        self._b = lib.lpcnet_batch_create(nb_streams, device)
        if not self._b:
            raise LPCNetError(f"lpcnet_batch_create failed: {last_error()}")
        self._owner = _BatchOwner(self._b)
        self.B = nb_streams
        if blob is not None:
            self.load_model(blob)

    def load_model(self, blob: bytes) -> None:
        if lib.lpcnet_batch_load_model(self._b, blob, len(blob)) != 0:
            raise LPCNetError(f"lpcnet_batch_load_model failed: {last_error()}")

    def set_kernel(self, mode: int) -> None:
        """0 automatic, 1 lockstep sample kernel, 4 mf_kernel (matrix cores), 5 fp_kernel (fp32);
        a mode the model cannot run falls back to 1."""
        if lib.lpcnet_batch_set_kernel(self._b, mode) != 0:
            raise LPCNetError(last_error())

    def set_model_constants(self, lpc_gamma: float = 1.0, features_delay: int = 2, end2end: bool = False) -> None:
        """LPC_GAMMA / FEATURES_DELAY / END2END of the loaded model (the reference's
        nnet_data.h constants); see lpcnet_batch_set_model_constants."""
        if lib.lpcnet_batch_set_model_constants(self._b, lpc_gamma, features_delay, 1 if end2end else 0) != 0:
            raise LPCNetError(last_error())

    def set_rcp_table(self, table: np.ndarray | None) -> None:
        """Same-box parity: the rcpps table of the device activations (4096
        entries, see host_rcp_table; None = the default Intel table)."""
        t = None if table is None else np.ascontiguousarray(table, np.uint32)
        if t is not None and t.size != 4096:
            raise ValueError("rcpps table must have 4096 entries (top 12 mantissa bits, see host_rcp_table); "
                             f"got {t.size}")
        if lib.lpcnet_batch_set_rcp_table(self._b, None if t is None else t.ctypes.data) != 0:
            raise LPCNetError(last_error())

    def set_spin_limit(self, polls: int) -> None:
        """LDS flag-wait bound of the barrier-free kernel (0 = default); see lpcnet_mi355x.h."""
        if lib.lpcnet_batch_set_spin_limit(self._b, polls) != 0:
            raise LPCNetError("bad spin limit")

    def set_frame_chunking(self, enable: bool) -> None:
        """Chunked frame network for batches above 128 streams (default on); off = per-frame kernel."""
        if lib.lpcnet_batch_set_frame_chunking(self._b, 1 if enable else 0) != 0:
            raise LPCNetError("set_frame_chunking failed")

    def info(self) -> ModelInfo:
        mi = ModelInfo()
        if lib.lpcnet_batch_model_info(self._b, C.byref(mi)) != 0:
            raise LPCNetError("no model loaded")
        return mi

    def reset(self, stream: int | None = None) -> None:
        if stream is None:
            lib.lpcnet_batch_reset(self._b)
        elif lib.lpcnet_batch_reset_stream(self._b, stream) != 0:
            raise LPCNetError(last_error())

    def synthesize(self, features: np.ndarray, n: int = FRAME_SIZE) -> np.ndarray:
        """features [B, >=20] -> pcm [B, n] int16 (one frame per stream)."""
        f = np.ascontiguousarray(np.asarray(features, np.float32)[:, :NB_FEATURES])
        assert f.shape[0] == self.B
        out = np.zeros((self.B, n), np.int16)
        if lib.lpcnet_batch_synthesize(self._b, f.ctypes.data, out.ctypes.data, n) != 0:
            raise LPCNetError(last_error())
        return out

    def host_features(self) -> np.ndarray:
        """The batch's feature buffer [B, 20] (lpcnet_batch_host_features:
        host-visible VRAM on large-BAR devices, else pinned host memory;
        write-combined there, so fill it in place and do not read it back
        in a hot loop), then synthesize_host()."""
        if getattr(self, "_hf", None) is None:
            p = lib.lpcnet_batch_host_features(self._b)
            if not p:
                raise LPCNetError(last_error())
            self._hf = _owned_view(self._owner, C.cast(p, C.c_void_p).value, C.c_float, np.float32, (self.B, NB_FEATURES))
            q = lib.lpcnet_batch_host_pcm(self._b)
            if not q:
                raise LPCNetError(last_error())
            self._hp = _owned_view(self._owner, C.cast(q, C.c_void_p).value, C.c_int16, np.int16, (self.B * FRAME_SIZE,))
            # the live tick's arguments, resolved once (ctypes attribute
            # lookups per call are microseconds of host turn-around)
            self._hf_addr, self._hp_addr = self._hf.ctypes.data, self._hp.ctypes.data
        return self._hf

    def synthesize_host(self, n: int = FRAME_SIZE) -> np.ndarray:
        """One frame from host_features() into the batch's pinned PCM buffer
        (lpcnet_batch_synthesize on the batch's own buffers: no host staging
        copies; the sample kernel stores the PCM there itself where it can).
        Returns a [B, n] view of that buffer, overwritten by the next call
        (copy it to keep it); the view keeps the batch's host buffers alive
        past close()."""
        self.host_features()
        if lib.lpcnet_batch_synthesize(self._b, self._hf_addr, self._hp_addr, n) != 0:
            raise LPCNetError(last_error())
        return self._hp[:self.B * n].reshape(self.B, n)

    def synthesize_impl(self, features: np.ndarray, pcm: np.ndarray, preload: int) -> np.ndarray:
        """lpcnet_synthesize_impl: pcm [B, N] int16, first ``preload`` samples teacher-forced."""
        f = np.ascontiguousarray(np.asarray(features, np.float32)[:, :NB_FEATURES])
        out = np.ascontiguousarray(pcm, np.int16).copy()
        n = out.shape[1] if out.ndim == 2 else 0
        if lib.lpcnet_batch_synthesize_impl(self._b, f.ctypes.data, out.ctypes.data if n else None, n, preload) != 0:
            raise LPCNetError(last_error())
        return out

    def frame_only(self, features: np.ndarray) -> None:
        """run_frame_network without samples (lpcnet.c:134 run_frame_network_flush)."""
        f = np.ascontiguousarray(np.asarray(features, np.float32)[:, :NB_FEATURES])
        if lib.lpcnet_batch_synthesize_impl(self._b, f.ctypes.data, None, 0, 0) != 0:
            raise LPCNetError(last_error())

    def synthesize_tail_impl(self, pcm: np.ndarray, preload: int = 0) -> np.ndarray:
        """lpcnet_synthesize_tail_impl on every stream: pcm [B, N] (first ``preload`` teacher-forced)."""
        out = np.ascontiguousarray(pcm, np.int16).copy()
        n = out.shape[1]
        if lib.lpcnet_batch_synthesize_tail_impl(self._b, out.ctypes.data if n else None, n, preload) != 0:
            raise LPCNetError(last_error())
        return out

    def run_frame_network(self, features: np.ndarray, update_conditions: bool) -> None:
        """run_frame_network of one frame per stream; update_conditions False = flush semantics."""
        f = np.ascontiguousarray(np.asarray(features, np.float32)[:, :NB_FEATURES])
        if lib.lpcnet_batch_run_frame_network(self._b, f.ctypes.data, 1 if update_conditions else 0) != 0:
            raise LPCNetError(last_error())

    def reset_signal(self, stream: int) -> None:
        if lib.lpcnet_batch_reset_signal(self._b, stream) != 0:
            raise LPCNetError(last_error())

    def decode(self, packets: np.ndarray) -> np.ndarray:
        """lpcnet_decode on every stream: packets [B, 8] uint8 -> pcm [B, 640]."""
        pk = np.ascontiguousarray(packets, np.uint8)
        assert pk.shape == (self.B, 8)
        out = np.zeros((self.B, 4 * FRAME_SIZE), np.int16)
        if lib.lpcnet_batch_decode(self._b, pk.ctypes.data, out.ctypes.data) != 0:
            raise LPCNetError(last_error())
        return out

    def decode_frames(self, d_packets: int, d_pcm: int, npackets: int) -> None:
        """Enqueue device packets [npackets, B, 8] -> device pcm [4 npackets, B, 160]."""
        if lib.lpcnet_batch_decode_frames(self._b, d_packets, d_pcm, npackets) != 0:
            raise LPCNetError(last_error())

    def save_state(self, stream: int) -> bytes:
        buf = C.create_string_buffer(lib.lpcnet_batch_state_size())
        if lib.lpcnet_batch_save_state(self._b, stream, buf) != 0:
            raise LPCNetError(last_error())
        return buf.raw

    def restore_state(self, stream: int, state: bytes) -> None:
        if lib.lpcnet_batch_restore_state(self._b, stream, state) != 0:
            raise LPCNetError(last_error())

    # -- device-resident path (benchmarks) ---------------------------------
    def device_alloc(self, nbytes: int) -> int:
        p = lib.lpcnet_batch_device_alloc(self._b, nbytes)
        if not p:
            raise LPCNetError(last_error())
        return p

    def device_free(self, p: int) -> None:
        lib.lpcnet_batch_device_free(self._b, p)

    def h2d(self, dst: int, arr: np.ndarray) -> None:
        a = np.ascontiguousarray(arr)
        if lib.lpcnet_batch_memcpy_h2d(self._b, dst, a.ctypes.data, a.nbytes) != 0:
            raise LPCNetError(last_error())

    def d2h(self, arr: np.ndarray, src: int) -> None:
        if lib.lpcnet_batch_memcpy_d2h(self._b, arr.ctypes.data, src, arr.nbytes) != 0:
            raise LPCNetError(last_error())

    def synthesize_frames(self, h_features: np.ndarray, d_features: int, d_pcm: int, nframes: int,
                          n: int = FRAME_SIZE) -> None:
        """Enqueue ``nframes`` frames from device features [nframes, B, 20] into device pcm
        [nframes, B, n].  ``h_features`` is unused (LPC runs on the device); kept for callers."""
        if lib.lpcnet_batch_synthesize_frames(self._b, None, d_features, d_pcm, nframes, n) != 0:
            raise LPCNetError(last_error())

    def sync(self) -> None:
        if lib.lpcnet_batch_sync(self._b) != 0:
            raise LPCNetError(last_error())

    def reset_timers(self, enable: bool | int = True) -> None:
        """0/False off, 1 sample kernel only, 2/True sample and frame kernels."""
        lib.lpcnet_batch_reset_timers(self._b, 2 if enable is True else int(enable))

    def kernel_ms(self, which: int = 0) -> tuple[float, int]:
        """(total ms, launches) of the timed launches since reset_timers."""
        n = C.c_int(0)
        ms = lib.lpcnet_batch_kernel_ms(self._b, which, C.byref(n))
        return ms, n.value

    def kernel_frames(self, which: int = 0) -> int:
        """Frames covered by the timed launches (multi-frame launches count each frame)."""
        return lib.lpcnet_batch_kernel_frames(self._b, which)

    def set_stamps(self, enable: bool = True) -> None:
        if lib.lpcnet_batch_set_stamps(self._b, 1 if enable else 0) != 0:
            raise LPCNetError(last_error())

    def get_stamps(self) -> np.ndarray:
        """[workgroups, 8 waves, 16] s_memtime sums of the last sample-kernel launch."""
        out = np.zeros((self.B, 8, 16), np.uint64)
        g = lib.lpcnet_batch_get_stamps(self._b, out.ctypes.data)
        if g < 0:
            raise LPCNetError("stamps not enabled")
        return out[:g]

    def get_frame_stamps(self) -> np.ndarray:
        """[workgroups, 16] s_memtime phase durations of the last frame-kernel launch."""
        out = np.zeros((self.B, 16), np.uint64)  # >= the frame kernel's workgroups for any batch
        g = lib.lpcnet_batch_get_frame_stamps(self._b, out.ctypes.data)
        if g < 0:
            raise LPCNetError("stamps not enabled")
        return out[:g]

    def set_trace(self, enable: bool = True) -> None:
        lib.lpcnet_batch_set_trace(self._b, 1 if enable else 0)

    def get_trace(self, n: int) -> tuple[np.ndarray, np.ndarray]:
        logits = np.zeros((self.B, n, 8), np.float32)
        exc = np.zeros((self.B, n), np.int32)
        if lib.lpcnet_batch_get_trace(self._b, logits.ctypes.data, exc.ctypes.data) != 0:
            raise LPCNetError("trace not enabled")
        return logits, exc

    def get_state(self, stream: int) -> dict:
        a = np.zeros(1152, np.float32)
        b = np.zeros(48, np.float32)
        lpc = np.zeros(16, np.float32)
        sa = np.zeros(384, np.float32)
        sb = np.zeros(16, np.float32)
        fc = C.c_int(0)
        if lib.lpcnet_batch_get_state(self._b, stream, a.ctypes.data, b.ctypes.data, lpc.ctypes.data,
                                      sa.ctypes.data, sb.ctypes.data, C.byref(fc)) != 0:
            raise LPCNetError(last_error())
        return {"gru_a_cond": a, "gru_b_cond": b, "lpc": lpc, "gru_a_state": sa, "gru_b_state": sb,
                "frame_count": fc.value}

    def close(self) -> None:
        """Release the batch: destroyed now, or when the last array handed
        out by host_features() / synthesize_host() goes."""
        if self._b:
            self._hf = self._hp = None
            self._b = None
            self._owner = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
