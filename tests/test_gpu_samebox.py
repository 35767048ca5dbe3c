"""Same-box parity (hard part 1): the reference's PCM
depends on the CPU it runs on through _mm256_rcp_ps (vec_avx.h:408,437).
The golden fixtures pin the Intel build host's; the GPU box's host is an AMD
EPYC whose rcpps is a different, 12-bit table (profiles/r03/box_rcpps.json).
Here the reference's own compiled kernels (oracle/_ref: vec_avx.h, kiss99.c,
freq.c, ... built from the reference sources) run LIVE on this box's CPU,
driven by the oracle's lpcnet.c/nnet.c restatement, and the engine with this
host's rcpps table (lpcnet_batch_set_rcp_table) must reproduce them bit for
bit -- PCM identical, every sample.  On an Intel host the two tables agree
and the engine's default kernels are used."""
import numpy as np
import pytest

import lpcnet_amd as L
import oracle_lib as O

pytestmark = pytest.mark.gpu


def feats(stream, nframes):
    return L.synthetic_features(stream, nframes)[:, :20]


@pytest.mark.skipif(not O.have_ref(), reason="oracle/_ref (the reference's compiled kernels) not built")
@pytest.mark.parametrize("variant", [0, 1])
def test_engine_with_host_rcpps_matches_live_reference(require_gpu, variant):
    tab, bad = L.host_rcp_table()
    assert bad == 0, "this host's rcpps is not a 12-bit exponent-invariant table"
    intel = np.array_equal(tab[::2], L.rcp_table()) and np.array_equal(tab[1::2], L.rcp_table())
    blob = L.synthetic_model(1, variant)
    B, F = 3, 14
    allf = np.stack([feats(s, F) for s in range(B)], 1)
    b = L.LPCNetBatch(B, 0, blob)
    b.set_rcp_table(tab)
    if not intel:
        assert b.info().quad_path in (0, 1)  # every activation through the table
    refs = [O.Oracle(blob, variant, O.ref_kernels()) for _ in range(B)]  # live reference kernels, this CPU
    ports = [O.Oracle(blob, variant) for _ in range(B)]                  # the Intel table (golden numerics)
    differ = 0
    for f in range(F):
        out = b.synthesize(allf[f])
        for s in range(B):
            exp = refs[s].synthesize(allf[f, s])
            assert np.array_equal(out[s], exp), (f, s)
            differ += int(np.sum(exp != ports[s].synthesize(allf[f, s])))
    print(f"host rcpps {'equals' if intel else 'differs from'} the Intel table; the live reference differs from "
          f"the Intel-table reference in {differ} of {B * F * 160} samples")
    if not intel and variant == 0:
        # the int8 model's PCM visibly depends on the host (the fp32 one may
        # not flip a sample in 14 frames: a rcpps difference changes a
        # logit's last bits, rarely a decision)
        assert differ > 0
    # back to the default table: the Intel-table numerics of the golden fixtures
    b.set_rcp_table(None)
    assert b.info().quad_path in ((5,) if variant else (4,))
