"""GPU parity of the GAE + normalisation kernels vs the NumPy oracle (fp32, 1e-5 relative)."""
import numpy as np
import pytest
import torch

from oracle import mappo as om

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("T,B,A", [(1, 1, 1), (7, 13, 2), (32, 4096, 25), (512, 128, 5), (64, 1000, 1)])
def test_gae_matches_oracle(T, B, A):
    from marlsat.learners.ops import gae

    rng = np.random.default_rng(T * 1000 + B)
    r = (rng.random((T, B, A)) < 0.05).astype(np.float32) * rng.standard_normal((T, B, A)).astype(np.float32)
    v = rng.standard_normal((T, B)).astype(np.float32)
    d = rng.random((T, B)) < 0.1
    lv = rng.standard_normal(B).astype(np.float32)
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    adv_raw, tgt = gae(cu(r), cu(v), cu(d), cu(lv), 0.995, 0.95, normalize=False)
    oadv, otgt = om.gae(r[..., 0], v, d, lv, 0.995, 0.95)
    # same op order, no contraction: bitwise
    np.testing.assert_array_equal(adv_raw.cpu().numpy(), oadv)
    np.testing.assert_array_equal(tgt.cpu().numpy(), otgt)
    adv, _ = gae(cu(r), cu(v), cu(d), cu(lv), 0.995, 0.95, normalize=True)
    if T * B > 1:
        onorm, _, _ = om.normalize(oadv)
        np.testing.assert_allclose(adv.cpu().numpy(), onorm, rtol=1e-5, atol=1e-6)
