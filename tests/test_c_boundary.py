"""The drop-in boundary from C: tools/lpcnet_synth.c is the `-synthesis` mode
of the reference demo (src/lpcnet_demo.c:202-219) written against
include/lpcnet.h only, built as plain C99 with -Werror and linked to
liblpcnet_mi355x.so.  The -m gpu test runs it on the golden stream's feature
file and byte-compares the PCM file with the fixture made from the
reference's own kernels (tests/golden/streams_int8.npz)."""
import os
import subprocess

import numpy as np
import pytest

import lpcnet_amd as L
import oracle_lib as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tools", "lpcnet_synth")


def _exe():
    if not os.path.exists(EXE):
        subprocess.run(["make", "-C", ROOT, "synth"], check=True, capture_output=True)
    return EXE


def test_header_is_plain_c_and_caller_links(tmp_path):
    """include/lpcnet.h compiles as strict C89/C99/C11 and the caller links."""
    for std in ("c89", "c99", "c11"):
        src = tmp_path / "h.c"
        src.write_text('#include "lpcnet.h"\n#include "lpcnet_mi355x.h"\nint main(void){return lpcnet_get_size() > 0 ? 0 : 1;}\n')
        exe = tmp_path / ("h_" + std)
        subprocess.run(["cc", "-std=" + std, "-pedantic", "-Wall", "-Werror", "-Wno-long-long",
                        "-I" + os.path.join(ROOT, "include"), "-o", str(exe), str(src),
                        "-L" + os.path.join(ROOT, "lpcnet_amd"), "-llpcnet_mi355x",
                        "-Wl,-rpath," + os.path.join(ROOT, "lpcnet_amd")], check=True)
        assert subprocess.run([str(exe)]).returncode == 0
    r = subprocess.run([_exe()], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr


def test_caller_fails_cleanly_without_device(tmp_path):
    if L.device_count() > 0:
        pytest.skip("a device is visible: covered by the -m gpu test")
    w = tmp_path / "w.bin"
    w.write_bytes(L.synthetic_model(1, 0))
    f = tmp_path / "f.f32"
    L.synthetic_features(0, 2).tofile(f)
    r = subprocess.run([_exe(), str(w), str(f), str(tmp_path / "o.pcm")], capture_output=True, text=True)
    assert r.returncode == 1 and "lpcnet_load_model failed" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("name,variant", [("streams_int8", 0), ("streams_fp32", 1)])
def test_c_caller_pcm_file_matches_golden(require_gpu, tmp_path, name, variant):
    G = np.load(os.path.join(O.GOLDEN, name + ".npz"))
    w = tmp_path / "weights.bin"
    w.write_bytes(L.synthetic_model(1, variant))
    f = tmp_path / "features.f32"
    feats = np.ascontiguousarray(G["features"][0], np.float32)  # [40][36], as lpcnet_demo -features writes
    assert feats.shape[1] == L.NB_TOTAL_FEATURES
    feats.tofile(f)
    out = tmp_path / "out.pcm"
    r = subprocess.run([_exe(), str(w), str(f), str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert out.read_bytes() == np.ascontiguousarray(G["pcm"][0], np.int16).tobytes()
    # a trailing partial frame is ignored, as the reference demo does (lpcnet_demo.c:212)
    with open(f, "ab") as fh:
        fh.write(b"\0" * 40)
    r = subprocess.run([_exe(), str(w), str(f), str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and out.stat().st_size == 40 * 160 * 2
