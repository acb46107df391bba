"""GPU: the clause / var gathers (msat_clause_gather2, msat_var_gather2) against a float32 restatement
that adds the same terms in the same order, compared BITWISE: learner:66-79's A±ᵀ M and A± M as
signed-literal gathers (csrc/gnn_kernels.hip).  Odd row counts exercise the half-wave tails (two rows
per wave), H = 64 / 128 / 256 the lane-to-column maps, empty slots and rows with no entries the edges."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _graph(Nv, Nc, seed):
    rng = np.random.default_rng(seed)
    slots = np.full((Nc, 3), -1, np.int64)
    for c in range(Nc):
        k = rng.integers(0, 4)  # 0..3 literals (0: an empty clause row)
        vs = rng.choice(Nv, size=k, replace=False)
        slots[c, :k] = (vs << 1) | rng.integers(0, 2, k)
    cl, sl = np.nonzero(slots >= 0)
    vals = slots[cl, sl]
    var, neg = vals >> 1, vals & 1
    order = np.lexsort((cl, var))  # per var row: ascending clause row (the batch assembly's order)
    inc = ((cl[order] << 1) | neg[order]).astype(np.int32)
    ptr = np.zeros(Nv + 1, np.int64)
    np.add.at(ptr, var + 1, 1)
    return slots.astype(np.int32), np.cumsum(ptr).astype(np.int32), inc


def _clause_ref(Xp, Xn, slots, H, merged, old):
    W = H if merged else 2 * H
    out = np.zeros((len(slots), W), np.float32)
    for c, row in enumerate(slots):
        for half in ((0,) if merged else (0, 1)):
            acc = np.zeros(H, np.float32)
            for s in row:
                if s >= 0 and (merged or (s & 1) == half):
                    acc = acc + ((Xn if s & 1 else Xp)[s >> 1])
            out[c, half * H:(half + 1) * H] = acc
    return out + old if old is not None else out


def _var_ref(Yp, Yn, ptr, inc, H, old_p, old_n):
    P = np.zeros((len(ptr) - 1, H), np.float32)
    N = np.zeros_like(P)
    for v in range(len(ptr) - 1):
        ap, an = np.zeros(H, np.float32), np.zeros(H, np.float32)
        for e in inc[ptr[v]:ptr[v + 1]]:
            if e & 1:
                an = an + Yn[e >> 1]
            else:
                ap = ap + Yp[e >> 1]
        P[v], N[v] = ap, an
    if old_p is not None:
        P, N = P + old_p, N + old_n
    return P, N


@pytest.mark.parametrize("H", [64, 128, 256])
@pytest.mark.parametrize("Nv,Nc", [(37, 101), (8, 3)])
def test_gathers_bitwise_against_ordered_sums(H, Nv, Nc):
    from marlsat import _lib

    slots, ptr, inc = _graph(Nv, Nc, seed=H + Nv)
    rng = np.random.default_rng(5)
    f = lambda *sh: rng.standard_normal(sh).astype(np.float32)
    Xp, Xn, Yp, Yn = f(Nv, H), f(Nv, H), f(Nc, H), f(Nc, H)
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    dslots, dptr, dinc = cu(slots), cu(ptr), cu(inc)
    dXp, dXn, dYp, dYn = cu(Xp), cu(Xn), cu(Yp), cu(Yn)
    s = _lib.stream_ptr()
    # clause side, split [pos | neg] and merged accumulating
    G = torch.full((Nc, 2 * H), 7.0, device="cuda")
    _lib.check(_lib.lib.msat_clause_gather2(dXp.data_ptr(), dXn.data_ptr(), H, dslots.data_ptr(), G.data_ptr(),
                                            2 * H, Nc, H, 0, 0, s), "clause_gather2")
    assert np.array_equal(G.cpu().numpy(), _clause_ref(Xp, Xn, slots, H, False, None))
    old = f(Nc, H)
    Gm = cu(old.copy())
    _lib.check(_lib.lib.msat_clause_gather2(dXp.data_ptr(), dXn.data_ptr(), H, dslots.data_ptr(), Gm.data_ptr(),
                                            H, Nc, H, 1, 1, s), "clause_gather2 merged")
    assert np.array_equal(Gm.cpu().numpy(), _clause_ref(Xp, Xn, slots, H, True, old))
    # var side, assigned and accumulating
    Vp, Vn = torch.full((Nv, H), 7.0, device="cuda"), torch.full((Nv, H), 7.0, device="cuda")
    _lib.check(_lib.lib.msat_var_gather2(dYp.data_ptr(), dYn.data_ptr(), H, dptr.data_ptr(), dinc.data_ptr(),
                                         Vp.data_ptr(), Vn.data_ptr(), H, Nv, H, 0, s), "var_gather2")
    P, N = _var_ref(Yp, Yn, ptr, inc, H, None, None)
    assert np.array_equal(Vp.cpu().numpy(), P) and np.array_equal(Vn.cpu().numpy(), N)
    op, on = f(Nv, H), f(Nv, H)
    Vp, Vn = cu(op.copy()), cu(on.copy())
    _lib.check(_lib.lib.msat_var_gather2(dYp.data_ptr(), dYn.data_ptr(), H, dptr.data_ptr(), dinc.data_ptr(),
                                         Vp.data_ptr(), Vn.data_ptr(), H, Nv, H, 1, s), "var_gather2 acc")
    P, N = _var_ref(Yp, Yn, ptr, inc, H, op, on)
    assert np.array_equal(Vp.cpu().numpy(), P) and np.array_equal(Vn.cpu().numpy(), N)


def test_var_gather_rows_longer_than_one_entry_chunk():
    """A var row with more entries than a half-wave's 32-entry chunk (and a wave whose two rows have very
    different lengths): the chunk loop and the per-half entry counts."""
    from marlsat import _lib

    H, Nv, Nc = 128, 3, 150
    rng = np.random.default_rng(9)
    slots = np.full((Nc, 3), -1, np.int32)
    slots[:, 0] = (0 << 1) | rng.integers(0, 2, Nc)  # var 0 in every clause: 150 entries
    slots[:40, 1] = (1 << 1) | 1                     # var 1: 40 negative entries
    cl, sl = np.nonzero(slots >= 0)
    vals = slots[cl, sl].astype(np.int64)
    order = np.lexsort((cl, vals >> 1))
    inc = ((cl[order] << 1) | (vals[order] & 1)).astype(np.int32)
    ptr = np.zeros(Nv + 1, np.int64)
    np.add.at(ptr, (vals >> 1) + 1, 1)
    ptr = np.cumsum(ptr).astype(np.int32)
    Yp, Yn = rng.standard_normal((Nc, H)).astype(np.float32), rng.standard_normal((Nc, H)).astype(np.float32)
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    Vp, Vn = torch.empty(Nv, H, device="cuda"), torch.empty(Nv, H, device="cuda")
    dev = [cu(a) for a in (Yp, Yn, ptr, inc)]  # held until the kernel has run (no temporaries behind raw pointers)
    _lib.check(_lib.lib.msat_var_gather2(dev[0].data_ptr(), dev[1].data_ptr(), H, dev[2].data_ptr(),
                                         dev[3].data_ptr(), Vp.data_ptr(), Vn.data_ptr(), H, Nv, H, 0,
                                         _lib.stream_ptr()), "var_gather2")
    P, N = _var_ref(Yp, Yn, ptr, inc, H, None, None)
    assert np.array_equal(Vp.cpu().numpy(), P) and np.array_equal(Vn.cpu().numpy(), N)
