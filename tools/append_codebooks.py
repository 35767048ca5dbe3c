#!/usr/bin/env python3
"""Append the 1.6 kb/s decoder's ceps codebooks to a weight blob.

The reference compiles its decoder codebooks in (generated
src/ceps_codebooks.c, declared lpcnet_private.h:109-112, sizes
lpcnet_enc.c:109-119 / :709); this library reads them from the model blob
instead, as four extra WeightHead records (nnet.h:54-61), which the
reference's own synthesis parser ignores.  A stock reference blob carries
none, so a deployment that decodes packets appends them once:

    python3 tools/append_codebooks.py weights.bin codebooks.f32 out.bin

codebooks.f32: raw little-endian float32, in this order:
    ceps_codebook1       1024 x 17
    ceps_codebook2       1024 x 17
    ceps_codebook3       1024 x 17
    ceps_codebook_diff4  4096 x 18
(the arrays of ceps_codebooks.c, concatenated).  Existing codebook records in
the blob are replaced.
"""
import struct
import sys

import numpy as np

SHAPES = (("ceps_codebook1", 1024 * 17), ("ceps_codebook2", 1024 * 17), ("ceps_codebook3", 1024 * 17),
          ("ceps_codebook_diff4", 4096 * 18))
HEAD = 64


def records(blob: bytes):
    off = 0
    while off < len(blob):
        if len(blob) - off < HEAD:
            raise ValueError("trailing bytes shorter than a record header at offset %d" % off)
        size, block = struct.unpack_from("<ii", blob, off + 12)
        if size < 0 or block < size or block > len(blob) - off - HEAD:
            raise ValueError("malformed record at offset %d" % off)
        name = blob[off + 20:off + HEAD].split(b"\0")[0].decode("latin-1")
        yield name, blob[off:off + HEAD + block]
        off += HEAD + block


def record(name: str, payload: bytes) -> bytes:
    block = (len(payload) + 63) // 64 * 64
    h = bytearray(HEAD)
    h[0:4] = b"DNNw"
    struct.pack_into("<iiii", h, 4, 0, 0, len(payload), block)  # version 0, WEIGHT_TYPE_float
    h[20:20 + len(name)] = name.encode()
    return bytes(h) + payload + bytes(block - len(payload))


def append_codebooks(blob: bytes, codebooks: np.ndarray) -> bytes:
    cb = np.ascontiguousarray(codebooks, np.float32).ravel()
    need = sum(n for _, n in SHAPES)
    if cb.size != need:
        raise ValueError("codebook file holds %d floats, expected %d" % (cb.size, need))
    names = {n for n, _ in SHAPES}
    out = bytearray(b"".join(r for name, r in records(blob) if name not in names))
    off = 0
    for name, n in SHAPES:
        out += record(name, cb[off:off + n].tobytes())
        off += n
    return bytes(out)


def main(argv):
    if len(argv) != 4:
        print(__doc__)
        return 2
    blob = open(argv[1], "rb").read()
    cb = np.fromfile(argv[2], dtype="<f4")
    open(argv[3], "wb").write(append_codebooks(blob, cb))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
