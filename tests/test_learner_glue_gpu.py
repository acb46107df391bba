"""GPU: the learner glue kernels (learner_kernels.hip) -- the epoch permutation, the micro-batch row
gather and the cycle metrics -- against numpy on the same inputs (bit-exact for indices and copies,
fp64 sums to 1e-12 relative)."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N", [1, 2, 3, 7, 64, 1000, 32768, 100003])
def test_permutation_is_a_keyed_bijection(N):
    from marlsat import _lib

    s = _lib.stream_ptr()
    outs = []
    for seed, ctr in ((1, 0), (1, 0), (2, 0), (1, 1)):
        p = torch.empty(N, dtype=torch.int32, device="cuda")
        _lib.check(_lib.lib.msat_permutation(N, seed, ctr, p.data_ptr(), s), "perm")
        a = p.cpu().numpy()
        assert np.array_equal(np.sort(a), np.arange(N))  # a permutation of [0, N)
        outs.append(a)
    assert np.array_equal(outs[0], outs[1])  # deterministic in (seed, counter)
    if N >= 64:  # different keys give different orders, and the order is not the identity
        assert not np.array_equal(outs[0], outs[2]) and not np.array_equal(outs[0], outs[3])
        assert (outs[0] != np.arange(N)).mean() > 0.9


def test_permutation_mixes_uniformly():
    """Position statistics over many keys: every row lands in every quarter of the order ~uniformly."""
    from marlsat import _lib

    N, K = 256, 400
    counts = np.zeros((N, 4))
    p = torch.empty(N, dtype=torch.int32, device="cuda")
    for k in range(K):
        _lib.check(_lib.lib.msat_permutation(N, 12345 + k, 0, p.data_ptr(), _lib.stream_ptr()), "perm")
        a = p.cpu().numpy()
        counts[a, np.arange(N) * 4 // N] += 1
    frac = counts / K
    assert np.abs(frac - 0.25).max() < 0.15, np.abs(frac - 0.25).max()


def test_gather_rows_matches_indexing():
    from marlsat import _lib

    g = torch.Generator(device="cuda").manual_seed(0)
    T, B, V, A = 4, 50, 37, 5
    srcs = [torch.randint(0, 1000, (T, B), dtype=torch.int32, device="cuda", generator=g),
            torch.randint(0, 2, (T, B, V), dtype=torch.uint8, device="cuda", generator=g),
            torch.randint(0, 9, (T, B, A), dtype=torch.int32, device="cuda", generator=g),
            torch.randn(T, B, A, device="cuda", generator=g), torch.randn(T, B, device="cuda", generator=g)]
    idx = torch.randint(0, T * B, (77,), dtype=torch.int32, device="cuda", generator=g)
    outs = [torch.empty((77,) + tuple(t.shape[2:]), dtype=t.dtype, device="cuda") for t in srcs]
    n = len(srcs)
    src = (ctypes.c_void_p * n)(*[t.data_ptr() for t in srcs])
    dst = (ctypes.c_void_p * n)(*[t.data_ptr() for t in outs])
    rb = (ctypes.c_int32 * n)(*[t[0, 0].numel() * t.element_size() for t in srcs])
    _lib.check(_lib.lib.msat_gather_rows(idx.data_ptr(), 77, n, src, dst, rb, _lib.stream_ptr()), "gather")
    for t, o in zip(srcs, outs):
        assert torch.equal(o, t.reshape((T * B,) + tuple(t.shape[2:]))[idx.long()])


def test_cycle_metrics_match_numpy():
    from marlsat import _lib

    rng = np.random.default_rng(0)
    N = 32768 + 5
    reward = rng.normal(size=N).astype(np.float32)
    done = (rng.random(N) < 0.1).astype(np.uint8)
    solved = (rng.random(N) < 0.5).astype(np.uint8)
    unsat = rng.integers(0, 50, N).astype(np.int32)
    steps = rng.integers(0, 512, N).astype(np.int32)
    tg = rng.normal(size=N).astype(np.float32)
    vp = rng.normal(size=N).astype(np.float32)
    dev = [torch.from_numpy(a).cuda() for a in (reward, done, solved, unsat, steps, tg, vp)]
    out = torch.empty(9, dtype=torch.float64, device="cuda")
    _lib.check(_lib.lib.msat_cycle_metrics(N, *[t.data_ptr() for t in dev], out.data_ptr(), _lib.stream_ptr()),
               "metrics")
    dn = done.astype(np.float64)
    sv = (solved.astype(bool) & done.astype(bool)).astype(np.float64)
    t, d = tg.astype(np.float64), tg.astype(np.float64) - vp.astype(np.float64)
    ref = [reward.astype(np.float64).sum(), dn.sum(), sv.sum(), (unsat * dn).sum(), (steps * sv).sum(), t.sum(),
           (t * t).sum(), d.sum(), (d * d).sum()]
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("S", [0, 1, 5, 1023, 1024, 1025, 32768, 40001])
def test_graph_bases_match_cumsum(S):
    from marlsat import _lib

    rng = np.random.default_rng(S)
    n_inst = 37
    counts = [rng.integers(0, 3000, n_inst).astype(np.int32) for _ in range(3)]
    inst = rng.integers(0, n_inst, S).astype(np.int32)
    dc = [torch.from_numpy(c).cuda() for c in counts]
    di = torch.from_numpy(inst).cuda()
    bases = torch.empty((max(S, 1), 3), dtype=torch.int32, device="cuda")
    tot = torch.empty(3, dtype=torch.int32, device="cuda")
    _lib.check(_lib.lib.msat_graph_bases(S, di.data_ptr(), *[c.data_ptr() for c in dc], bases.data_ptr(),
                                         tot.data_ptr(), _lib.stream_ptr()), "graph_bases")
    per = np.stack([c[inst] for c in counts], 1).astype(np.int64)
    ref = np.cumsum(per, 0) - per
    assert np.array_equal(bases.cpu().numpy()[:S], ref)
    assert np.array_equal(tot.cpu().numpy(), per.sum(0))


def test_graph_bases_flag_int32_overflow():
    """A batch whose var-row total passes INT32_MAX gets the total -1 (not a clamped or wrapped
    count), and assemble-side callers refuse it."""
    from marlsat import _lib

    S = 3000
    counts = [np.full(2, 1_000_000, np.int32), np.full(2, 5, np.int32), np.full(2, 7, np.int32)]
    dc = [torch.from_numpy(c).cuda() for c in counts]
    di = torch.zeros(S, dtype=torch.int32, device="cuda")
    bases = torch.empty((S, 3), dtype=torch.int32, device="cuda")
    tot = torch.empty(3, dtype=torch.int32, device="cuda")
    _lib.check(_lib.lib.msat_graph_bases(S, di.data_ptr(), *[c.data_ptr() for c in dc], bases.data_ptr(),
                                         tot.data_ptr(), _lib.stream_ptr()), "graph_bases")
    assert tot.cpu().tolist() == [-1, 5 * S, 7 * S]


@pytest.mark.parametrize("V,C,vpa,S,micro", [(20, 91, 10, 77, 20), (50, 218, 10, 64, 64), (100, 430, 10, 33, 7)])
def test_batch_totals_match_the_device_totals(V, C, vpa, S, micro):
    """The learner's per-minibatch size plan (graphs.batch_totals, one device -> host read for all its
    micro-batches) equals what msat_graph_bases computes for each micro-batch, and a batch assembled
    with the planned totals is identical to one assembled with the device read."""
    from marlsat import SATEnv
    from marlsat.learners.graphs import DeviceTemplates, assemble, batch_totals, build_templates
    from marlsat.utils.generate_cnf_dataset import generate_problem_pool

    N = 16
    pool = generate_problem_pool(V, C, N, size_id=5)
    env = SATEnv(V, C, max_steps=10, vars_per_agent=vpa)
    A = env.num_agents
    dpool = env.make_pool(pool)
    tpl = DeviceTemplates(build_templates(pool, V, A), A, "cuda")
    rng = np.random.default_rng(V + S)
    inst = torch.from_numpy(rng.integers(0, N, S).astype(np.int32)).cuda()
    x = torch.from_numpy(rng.integers(0, 2, (S, V)).astype(np.uint8)).cuda()
    bounds = list(range(0, S, micro)) + [S]
    plan = batch_totals(tpl, inst, bounds)
    assert len(plan) == len(bounds) - 1
    svf = dpool.static_var_features()
    for (m0, m1), tot in zip(zip(bounds[:-1], bounds[1:]), plan):
        a = assemble(tpl, dpool.packed, svf, inst[m0:m1].contiguous(), x[m0:m1].contiguous())
        b = assemble(tpl, dpool.packed, svf, inst[m0:m1].contiguous(), x[m0:m1].contiguous(), totals=tot)
        assert (a.Nv, a.Nc, a.nnz) == tot
        for f in ("vfeat", "cfeat", "cdeg", "slots", "ptr", "inc", "vbase", "nv", "cbase", "nc"):
            assert torch.equal(getattr(a, f), getattr(b, f)), f
