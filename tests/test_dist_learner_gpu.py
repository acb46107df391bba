"""GPU: the device learner sharded over 2 ranks == the same learner on 1 rank over the union
(learner:530-532 global advantage normalisation, learner:647-650 one Adam step
per minibatch on its mean gradient).

A fresh child ``python -m torch.distributed.run`` (a subprocess, never an exec of this test
process) runs tests/dist_learner_worker.py with 2 ranks on this GPU over gloo
(MARLSAT_SHARE_GPU-style rehearsal: RCCL refuses two ranks per device; the driver's 8-GPU
runs use RCCL through the same learners/collectives.py calls).  This process runs the union
(world 1) and then, teacher-forced, recomputes each sharded Adam step's gradient on the union
of the two ranks' minibatch rows from the sharded run's own parameters.  Checks:
  * every rank holds bitwise identical parameters after every Adam step (replicas stay equal);
  * the globally normalised advantages and targets equal the union's (1e-6);
  * every step's all-reduced gradient (x 1/world) equals the union minibatch gradient,
    elementwise 1e-5 relative + 4x the tensor's fp32 reduction-order noise (the union gradient
    summed in one vs two micro-batches; the forward of a sample is row-local, so summation
    order is the only difference);
  * the loss triple every rank REPORTS for each minibatch (MAPPOLearner.metrics' arrays) is the
    union minibatch's, identical on both ranks, 1e-5 relative to the union run.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_learner_equals_union(tmp_path):
    import dist_learner_worker as W
    from marlsat.learners import params as Pm

    env = dict(os.environ, MARLSAT_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(HERE, "dist_learner_worker.py"),
           str(tmp_path)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    ranks = [torch.load(os.path.join(tmp_path, f"rank{k}.pt"), weights_only=True) for k in range(2)]
    # replicas stay identical
    assert torch.equal(ranks[0]["final"], ranks[1]["final"])
    assert torch.isfinite(ranks[0]["final"]).all()
    for a, b in zip(ranks[0]["trace"], ranks[1]["trace"]):
        assert torch.equal(a["params"], b["params"]) and torch.equal(a["grads"], b["grads"])
    # union run, world 1
    u = W.run(0, 1, None, minibatches_per_rank=2)
    learner = u.pop("learner")
    T, Bl = W.T, W.B_UNION // 2
    cat = lambda key: torch.cat([ranks[0][key], ranks[1][key]], 1)  # (T, Bl) shards -> (T, B_UNION)
    np.testing.assert_allclose(cat("adv").numpy(), u["adv"].numpy(), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(cat("targets").numpy(), u["targets"].numpy(), rtol=1e-6, atol=1e-7)
    net = learner.net
    # from here on the union evaluates every step on the sharded run's normalised advantages and targets
    # (equal to 1e-6 above): otherwise a ratio sitting within 1e-7 of the clip edge 1 +- eps could take
    # the other branch of min(r A, clip(r) A) and move a whole sample's actor gradient
    learner.adv.copy_(cat("adv").to(learner.adv.device))
    learner.targets.copy_(cat("targets").to(learner.targets.device))
    # the learner reports rank-global losses (learner:708-719): every rank holds the union minibatch's
    # triple itself, identical on both ranks (one all-reduce of the row sums per cycle)
    assert torch.equal(ranks[0]["losses"], ranks[1]["losses"])
    losses_sharded = ranks[0]["losses"]
    for s, rec in enumerate(ranks[0]["trace"]):
        rows = []
        for k in range(2):
            li = ranks[k]["trace"][s]["idx"].numpy()
            t, b = li // Bl, li % Bl
            rows.append(t * W.B_UNION + k * Bl + b)  # local flat row -> union flat row
        idx = torch.from_numpy(np.concatenate(rows)).to(net.device)
        net.params.copy_(rec["params"].to(net.device))
        # the same union gradient summed in two micro-batches instead of one: its difference from the
        # one-pass sum is the fp32 reduction-order noise of each tensor (the embeddings' gradients sum
        # thousands of rows with heavy cancellation), the yardstick of the sharded-vs-union check
        micro = learner.micro
        learner.micro = (idx.numel() + 1) // 2
        learner.minibatch_grad(idx, float(W.CFG["ENT_COEF"]), torch.zeros(3, dtype=torch.float64,
                                                                            device=net.device), idx.numel())
        alt = Pm.to_flax(net.grads.cpu().numpy(), net.H, net.L, net.A, net.M, net.mode, net.E)
        learner.micro = idx.numel()
        sums = torch.zeros(3, dtype=torch.float64, device=net.device)
        learner.minibatch_grad(idx, float(W.CFG["ENT_COEF"]), sums, idx.numel())
        learner.micro = micro
        ref = Pm.to_flax(net.grads.cpu().numpy(), net.H, net.L, net.A, net.M, net.mode, net.E)
        got = Pm.to_flax(rec["grads"].numpy(), net.H, net.L, net.A, net.M, net.mode, net.E)
        for name in ref:
            g, r_, a_ = (t[name].astype(np.float64) for t in (got, ref, alt))
            noise = np.abs(a_ - r_).max()
            np.testing.assert_allclose(g, r_, rtol=1e-5, atol=4.0 * noise + 1e-9 * max(np.abs(r_).max(), 1e-30),
                                       err_msg=f"step {s} grad {name} (reduction noise {noise:.2e})")
        A = net.A
        s_ = sums.cpu().numpy() / np.array([idx.numel(), idx.numel() * A, idx.numel() * A])
        e, k = divmod(s, losses_sharded.shape[1])
        np.testing.assert_allclose(losses_sharded[e, k].numpy(), s_, rtol=1e-5, atol=1e-8, err_msg=f"step {s}")


@pytest.mark.parametrize("H", [64, 128])
def test_two_rank_train_cycles_keep_replicas_identical(tmp_path, H):
    """The bench's path at 2 ranks (own env shards and rollouts, two full train cycles, gradient
    all-reduce before every Adam step): every Adam step starts from bitwise identical parameters on both
    ranks and applies a bitwise identical all-reduced gradient, at H = 64 (fp32 kernels) and H = 128
    (fp16x2 / bf16x3 kernels)."""
    env = dict(os.environ, MARLSAT_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(HERE, "dist_replica_worker.py"),
           str(tmp_path), str(H)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    ranks = [torch.load(os.path.join(tmp_path, f"rank{k}.pt"), weights_only=True) for k in range(2)]
    assert torch.equal(ranks[0]["init"], ranks[1]["init"])
    assert len(ranks[0]["trace"]) == len(ranks[1]["trace"]) > 0
    for s, (a, b) in enumerate(zip(ranks[0]["trace"], ranks[1]["trace"])):
        assert torch.equal(a["params"], b["params"]), f"Adam step {s}: parameters differ across ranks"
        assert torch.equal(a["grads"], b["grads"]), f"Adam step {s}: all-reduced gradients differ across ranks"
    assert torch.equal(ranks[0]["final"], ranks[1]["final"])
    assert torch.isfinite(ranks[0]["final"]).all()
