"""GPU: categorical sampling (distrax.Categorical sample / log_prob, learner:397-403) by the
Gumbel-max kernel -- empirical frequencies vs softmax, masked (-inf) actions never drawn,
log-probs exact, greedy = first argmax (jnp.argmax ties), counter-based reproducibility."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _sample(logits, greedy, seed, counter):
    from marlsat import _lib

    R, W = logits.shape
    act = torch.empty(R, dtype=torch.int32, device="cuda")
    lp = torch.empty(R, dtype=torch.float32, device="cuda")
    _lib.check(_lib.lib.msat_sample_actions(logits.data_ptr(), R, W, 1 if greedy else 0, seed, counter,
                                            act.data_ptr(), lp.data_ptr(), _lib.stream_ptr()), "sample")
    torch.cuda.synchronize()
    return act, lp


@pytest.mark.parametrize("W", [2, 9, 11, 70])
def test_gumbel_sampling_statistics(W):
    R = 200000
    g = torch.Generator(device="cuda").manual_seed(W)
    row = torch.randn(W, device="cuda", generator=g) * 1.5
    masked = W // 2 if W > 2 else -1  # a masked action (W = 2 keeps both: two outcomes needed below)
    if masked >= 0:
        row[masked] = float("-inf")
    logits = row.expand(R, W).contiguous()
    act, lp = _sample(logits, False, 1234, 7)
    a = act.long().cpu()
    assert int(a.min()) >= 0 and int(a.max()) < W and not bool((a == masked).any())
    p = torch.softmax(row.double().cpu(), 0)
    freq = torch.bincount(a, minlength=W).double() / R
    sigma = (p * (1 - p) / R).sqrt()
    assert bool(((freq - p).abs() <= 5 * sigma + 1e-12).all()), (freq, p)
    ref_lp = torch.log_softmax(row.double(), 0)[act.long()].float()
    assert torch.allclose(lp, ref_lp, rtol=0, atol=2e-6)
    act2, _ = _sample(logits, False, 1234, 7)
    act3, _ = _sample(logits, False, 1234, 8)
    assert torch.equal(act, act2) and not torch.equal(act, act3)


def test_greedy_argmax_first_tie_and_masks():
    lg = torch.tensor([[0.5, 2.0, 2.0, -1.0], [float("-inf"), -3.0, -3.0, float("-inf")],
                       [float("-inf")] * 3 + [0.0], [7.0, 7.0, 7.0, 7.0]], device="cuda")
    act, lp = _sample(lg, True, 0, 0)
    assert act.tolist() == [1, 1, 3, 0]
    assert torch.allclose(lp, torch.log_softmax(lg.double(), 1).gather(1, act.long()[:, None])[:, 0].float())
