"""ctypes wrapper of the CPU checker (oracle/liblpcnet_oracle.so and, when
built, oracle/_ref/libref_kernels.so).  TEST INFRASTRUCTURE ONLY."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liblpcnet_oracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_kernels.so")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def ensure_built():
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)


ORACLE_AVX2_SO = os.path.join(ROOT, "oracle", "liblpcnet_oracle_avx2.so")

ensure_built()
_vp, _i = C.c_void_p, C.c_int
_SIGS = [
    ("oracle_port_kernels", _vp, []),
    ("oracle_set_rcp_table", None, [_vp]),
    ("oracle_rcp", C.c_float, [C.c_float]),
    ("oracle_tanh", C.c_float, [C.c_float]),
    ("oracle_sigmoid", C.c_float, [C.c_float]),
    ("oracle_quantize_u8", None, [_vp, _vp, _i]),
    ("oracle_create", _vp, [C.c_char_p, _i, _i, _vp]),
    ("oracle_destroy", None, [_vp]),
    ("oracle_reset", None, [_vp]),
    ("oracle_synthesize", None, [_vp, _vp, _vp, _i, _i]),
    ("oracle_set_trace", None, [_vp, _vp, _vp, _vp]),
    ("oracle_set_constants", _i, [_vp, C.c_float, _i, _i]),
    ("oracle_get_frame", None, [_vp, _vp, _vp, _vp]),
    ("oracle_frame_count", _i, [_vp]),
    ("oracle_get_state", None, [_vp, _vp, _vp]),
    ("oracle_synthesize_tail", None, [_vp, _vp, _i, _i]),
    ("oracle_frame_deferred", None, [_vp, _vp]),
    ("oracle_frame_flush", None, [_vp]),
    ("oracle_reset_signal", None, [_vp]),
    ("oracle_state_size", _i, []),
    ("oracle_state_save", None, [_vp, _vp]),
    ("oracle_state_restore", None, [_vp, _vp]),
    ("oracle_decode_packet", _i, [_vp, _vp, _vp]),
    ("oracle_decode", _i, [_vp, _vp, _vp]),
]
RCP_TABLE = np.fromfile(os.path.join(GOLDEN, "rcp_x86.bin"), dtype=np.uint32)
assert RCP_TABLE.size == 2048


def _bind(path):
    lib = C.CDLL(path)
    for name, res, args in _SIGS:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    lib.oracle_set_rcp_table(RCP_TABLE.ctypes.data)
    return lib


_ora = _bind(ORACLE_SO)
# the same restatement under the reference's -O3 -mavx2 -mfma flags: the CPU
# baseline's build (bench.py cpu_baseline), bit-identical (tests/test_oracle.py)
_ora_avx2 = _bind(ORACLE_AVX2_SO) if os.path.exists(ORACLE_AVX2_SO) else None


def have_avx2_build() -> bool:
    return _ora_avx2 is not None

_ref = None
if os.path.exists(REF_SO):
    try:
        _ref = C.CDLL(REF_SO)
        _ref.ref_kernels.restype = _vp
        _ref.ref_rcp_table.restype = _i
        _ref.ref_rcp_table.argtypes = [_vp]
        _ref.ref_rcp.restype = C.c_float
        _ref.ref_rcp.argtypes = [C.c_float]
        _ref.ref_quantize_u8.argtypes = [_vp, _vp, _i]
    except OSError:
        _ref = None


def have_ref() -> bool:
    return _ref is not None


REF_PARSE = {0: os.path.join(ROOT, "oracle", "_ref", "ref_parse_int8"),
             1: os.path.join(ROOT, "oracle", "_ref", "ref_parse_fp32")}


def have_ref_parser() -> bool:
    return all(os.path.exists(p) for p in REF_PARSE.values())


def ref_parse(blob: bytes, variant: int = 0, timeout: float = 5.0):
    """Run the reference's own parse_weights + layer binders
    (parse_lpcnet_weights.c, compiled unmodified by oracle/Makefile, driven by
    oracle/ref_parse.c) on ``blob`` in a fresh process.  Returns (outcome,
    bound): outcome "accept", "reject" (a binder refused), "parse_reject"
    (parse_weights refused), "hang" (killed at the timeout: find_idx_check's
    nb = -1 loop) or "crash" (killed by a signal); bound = {array name:
    (offset into the blob, bytes)} of the arrays the binders took."""
    try:
        r = subprocess.run([REF_PARSE[variant]], input=blob, capture_output=True, timeout=timeout)
    except subprocess.TimeoutExpired:
        return "hang", {}
    if r.returncode < 0:
        return "crash", {}
    outcome = {0: "accept", 1: "reject", 2: "parse_reject"}.get(r.returncode)
    if outcome is None:
        return "crash", {}
    bound = {}
    for line in r.stdout.decode().splitlines():
        name, off, n = line.split()
        bound[name] = (int(off), int(n))
    return outcome, bound


def port_kernels():
    return _ora.oracle_port_kernels()


def ref_kernels():
    return _ref.ref_kernels() if _ref is not None else None


def kernel_table(k: C.c_void_p):
    """Calls into an oracle_kernels table (struct of function pointers)."""
    FT = C.CFUNCTYPE
    vp, i = C.c_void_p, C.c_int

    class K(C.Structure):
        _fields_ = [
            ("vec_tanh", FT(None, vp, vp, i)),
            ("vec_sigmoid", FT(None, vp, vp, i)),
            ("tanh1", FT(C.c_float, C.c_float)),
            ("sgemv16", FT(None, vp, vp, i, i, i, vp)),
            ("sparse8x4_i8", FT(None, vp, vp, i, i, vp, vp)),
            ("dense8x4_i8", FT(None, vp, vp, i, i, vp)),
            ("sparse8x4_f32", FT(None, vp, vp, i, vp, vp)),
            ("lin2ulaw", FT(i, C.c_float)),
            ("ulaw2lin", FT(C.c_float, C.c_float)),
            ("rng_srand", FT(None, vp, vp, i)),
            ("rng_rand", FT(C.c_uint32, vp)),
            ("lpc_from_cepstrum", FT(C.c_float, vp, vp)),
            ("lpc_weighting", FT(None, vp, C.c_float)),
        ]

    return K.from_address(k)


class Oracle:
    """One reference-semantics synthesis stream on the CPU."""

    def __init__(self, blob: bytes, variant: int = 0, kernels=None, constants=None, avx2_build: bool = False):
        """constants: (LPC_GAMMA, FEATURES_DELAY, END2END) of the model, the
        #defines the reference compiles in from nnet_data.h; default (1.0, 2, 0).
        avx2_build: the -O3 -mavx2 -mfma build of the restatement (CPU baseline)."""
        lib = _ora_avx2 if avx2_build and _ora_avx2 is not None else _ora
        self._lib = lib
        self._st = lib.oracle_create(blob, len(blob), variant, kernels or lib.oracle_port_kernels())
        if not self._st:
            raise ValueError("oracle_create: blob rejected")
        if constants is not None:
            g, d, e = constants
            if self._lib.oracle_set_constants(self._st, g, int(d), int(e)) != 0:
                raise ValueError("oracle_set_constants: unsupported value")

    def synthesize(self, features: np.ndarray, n: int = 160, preload: np.ndarray | None = None,
                   trace: bool = False):
        f = np.ascontiguousarray(np.asarray(features, np.float32)[:20])
        out = np.zeros(max(n, 1), np.int16)
        npre = 0 if preload is None else min(len(preload), n)
        if npre:
            out[:npre] = np.asarray(preload, np.int16)[:npre]
        if trace:
            lg = np.zeros((n, 8), np.float32)
            ex = np.zeros(n, np.int32)
            rw = np.zeros((n, 2), np.uint32)
            self._lib.oracle_set_trace(self._st, lg.ctypes.data, ex.ctypes.data, rw.ctypes.data)
        self._lib.oracle_synthesize(self._st, f.ctypes.data, out.ctypes.data, n, npre)
        out = out[:n]
        if trace:
            self._lib.oracle_set_trace(self._st, None, None, None)
            return out, lg, ex, rw
        return out

    def synthesize_tail(self, pcm: np.ndarray, preload: int = 0) -> np.ndarray:
        """lpcnet_synthesize_tail_impl: pcm [N] (first ``preload`` teacher-forced)."""
        out = np.ascontiguousarray(pcm, np.int16).copy()
        self._lib.oracle_synthesize_tail(self._st, out.ctypes.data, out.size, preload)
        return out

    def frame_deferred(self, features: np.ndarray) -> None:
        f = np.ascontiguousarray(np.asarray(features, np.float32)[:20])
        self._lib.oracle_frame_deferred(self._st, f.ctypes.data)

    def frame_flush(self) -> None:
        self._lib.oracle_frame_flush(self._st)

    def reset_signal(self) -> None:
        self._lib.oracle_reset_signal(self._st)

    def save(self) -> bytes:
        buf = C.create_string_buffer(self._lib.oracle_state_size())
        self._lib.oracle_state_save(self._st, buf)
        return buf.raw

    def restore(self, state: bytes) -> None:
        self._lib.oracle_state_restore(self._st, state)

    def decode_packet(self, packet: bytes) -> np.ndarray:
        """decode_packet (lpcnet_dec.c:81-156): 8 bytes -> features [4, 36]."""
        f = np.zeros((4, 36), np.float32)
        if self._lib.oracle_decode_packet(self._st, bytes(packet), f.ctypes.data) != 0:
            raise ValueError("blob has no codebooks")
        return f

    def decode(self, packet: bytes) -> np.ndarray:
        """lpcnet_decode (lpcnet.c:310-319): 8 bytes -> pcm [640]."""
        out = np.zeros(640, np.int16)
        if self._lib.oracle_decode(self._st, bytes(packet), out.ctypes.data) != 0:
            raise ValueError("blob has no codebooks")
        return out

    def frame(self):
        a = np.zeros(1152, np.float32)
        b = np.zeros(48, np.float32)
        lpc = np.zeros(16, np.float32)
        self._lib.oracle_get_frame(self._st, a.ctypes.data, b.ctypes.data, lpc.ctypes.data)
        return a, b, lpc

    def state(self):
        a = np.zeros(384, np.float32)
        b = np.zeros(16, np.float32)
        self._lib.oracle_get_state(self._st, a.ctypes.data, b.ctypes.data)
        return a, b

    def frame_count(self) -> int:
        return self._lib.oracle_frame_count(self._st)

    def reset(self):
        self._lib.oracle_reset(self._st)

    def __del__(self):
        try:
            self._lib.oracle_destroy(self._st)
        except Exception:
            pass


def synth_stream(blob: bytes, feats: np.ndarray, variant: int = 0, kernels=None, n: int = 160,
                 constants=None) -> np.ndarray:
    o = Oracle(blob, variant, kernels, constants)
    return np.stack([o.synthesize(feats[f], n) for f in range(len(feats))])


def oracle_tanh(x: float) -> float:
    return _ora.oracle_tanh(x)


def oracle_sigmoid(x: float) -> float:
    return _ora.oracle_sigmoid(x)


def oracle_rcp(x: float) -> float:
    return _ora.oracle_rcp(x)


def ref_rcp(x: float) -> float:
    return _ref.ref_rcp(x)


def ref_rcp_table() -> tuple[np.ndarray, int]:
    t = np.zeros(2048, np.uint32)
    bad = _ref.ref_rcp_table(t.ctypes.data)
    return t, bad


def quantize_u8(x: np.ndarray, ref: bool = False) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32)
    out = np.zeros(len(x) + 32, np.uint8)
    (_ref.ref_quantize_u8 if ref else _ora.oracle_quantize_u8)(out.ctypes.data, x.ctypes.data, len(x))
    return out[:len(x)]
