"""GPU: the clause cell's GRU backward (msat_gru_ln_bwd_g4fe, nfeat 2: gru_ln_bwd_kernel<2,true,6,2>) pinned
bitwise through its two-stage partial reduction.

The kernel writes one row of column partials per block (part[b][q*H + j], q = the 12 partial rows: LN scale /
bias, the four gate biases, and the feature-weighted gate sums of the two count features).  colsum4_kernel
folds 16 block rows per split in a fixed order, partial_reduce4_kernel folds the splits in a fixed order into
the gradients (dln, dbi, dbh_n, dfeat).  This test reads the block partials back and replays both stages on
the host in fp32 in exactly that order: the gradients must match BITWISE, and the fp64 sum of the same
partials must agree to fp32 rounding.  Twenty launches on the same inputs must be bitwise identical (the
round-3 run-to-run difference sat in dF row 2H + 1 = dfeat row 1, columns 304-319 / 368-383: DESIGN.md §8).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

H, NQ, KPART = 128, 12, 16  # hidden width, partial rows of the clause cell (6 + 3 * 2), rows per colsum4 split


def _fold16(rows: np.ndarray) -> np.ndarray:
    """colsum4 / partial_reduce4 in fp32: lane ty sums rows ty, ty + 16, ... from 0 in order, then lane 0
    adds the 16 lane sums in order (numpy float32 scalar adds, no pairwise summation)."""
    n = rows.shape[0]
    lanes = []
    for ty in range(16):
        a = np.zeros(rows.shape[1], np.float32)
        for r in range(ty, n, 16):
            a = (a + rows[r]).astype(np.float32)
        lanes.append(a)
    t = lanes[0]
    for k in range(1, 16):
        t = (t + lanes[k]).astype(np.float32)
    return t


def test_clause_cell_backward_reduction_is_bitwise_fixed_order():
    from marlsat import _lib

    L = _lib.lib
    R = 60001  # > 1024 * 4 rows: the grid caps at 1024 blocks, each walking ~15 rows
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(11)
    dy = torch.randn(R, H, device=dev, generator=g)
    g4 = torch.randn(R, 4 * H, device=dev, generator=g)
    hp = torch.randn(R, H, device=dev, generator=g)
    sc = torch.randn(H, device=dev, generator=g)
    feat = torch.randint(0, 4, (R, 4), device=dev, generator=g).float()  # [n+, n-, 0, 0] literal counts
    part = torch.empty(int(L.msat_gru_ln_bwd_partial_floats(R, H)), device=dev)
    s = _lib.stream_ptr()

    def run(seed_grads):
        D = torch.empty(R, 4 * H, device=dev)
        dh = torch.empty(R, H, device=dev)
        dln = seed_grads[0].clone()
        dbi = seed_grads[1].clone()
        dbh = seed_grads[2].clone()
        dfeat = seed_grads[3].clone()
        rexp = torch.empty(R, dtype=torch.int32, device=dev)
        _lib.check(L.msat_gru_ln_bwd_g4fe(dy.data_ptr(), H, g4.data_ptr(), 4 * H, hp.data_ptr(), H, sc.data_ptr(),
                                          D.data_ptr(), 4 * H, D.data_ptr() + 4 * H, 4 * H, dh.data_ptr(), H,
                                          dln.data_ptr(), dln.data_ptr() + 4 * H, dbi.data_ptr(),
                                          dbh.data_ptr() + 4 * 2 * H, feat.data_ptr(), 4, 2, dfeat.data_ptr(),
                                          part.data_ptr(), R, H, 7, rexp.data_ptr(), s), "gru_ln_bwd_g4fe")
        return dln, dbi, dbh, dfeat

    # accumulating outputs start from non-zero gradients (dbi, dbh_n and dfeat add; dln is assigned: flags & 1 = 1
    # accumulates too) -- the replay adds in the same place
    seed = [torch.randn(2 * H, device=dev, generator=g), torch.randn(3 * H, device=dev, generator=g),
            torch.randn(3 * H, device=dev, generator=g), torch.randn(2, 3 * H, device=dev, generator=g)]
    outs = run(seed)
    torch.cuda.synchronize()
    nb = min((R + 3) // 4, 1024)
    blocks = part[:nb * NQ * H].view(nb, NQ * H).cpu().numpy()
    sp = (nb + KPART - 1) // KPART
    ws_dev = part[nb * NQ * H:(nb + sp) * NQ * H].view(sp, NQ * H).cpu().numpy()
    # stage 1: each split's 16 block rows (one row per lane, 0 + v), folded in order
    ws = np.stack([_fold16(blocks[y * KPART:min(nb, (y + 1) * KPART)]) for y in range(sp)])
    assert np.array_equal(ws.view(np.int32), ws_dev.view(np.int32)), "colsum4 stage"
    # stage 2: the splits folded in order, added to the seeded gradient
    tot = _fold16(ws)
    want = {"dln": tot[0:2 * H], "dbi": tot[2 * H:5 * H], "dbh": tot[5 * H:6 * H], "dfeat": tot[6 * H:12 * H]}
    base = [seed[0].cpu().numpy(), seed[1].cpu().numpy(), seed[2].cpu().numpy()[2 * H:], seed[3].cpu().numpy().ravel()]
    got = [outs[0].cpu().numpy(), outs[1].cpu().numpy(), outs[2].cpu().numpy()[2 * H:], outs[3].cpu().numpy().ravel()]
    for (name, w), b, o in zip(want.items(), base, got):
        ref = (b + w).astype(np.float32)
        assert np.array_equal(ref.view(np.int32), o.view(np.int32)), name
    # the fp64 sum of the same block partials: within the fp32 folding error
    exact = blocks.astype(np.float64).sum(0)
    err = np.abs(tot.astype(np.float64) - exact)
    bound = 2.0 ** -23 * (nb + 32) * np.abs(blocks.astype(np.float64)).sum(0)
    assert (err <= bound).all(), float((err / np.maximum(bound, 1e-300)).max())
    # n- feature row (dF row 2H + 1), the columns of the round-3 report, are non-trivial here
    assert np.abs(tot[11 * H + 48:11 * H + 64]).min() > 0 and np.abs(tot[11 * H + 112:12 * H]).min() > 0
    # run to run: bitwise identical
    for _ in range(20):
        again = run(seed)
        torch.cuda.synchronize()
        for a, b in zip(again, outs):
            assert torch.equal(a, b)
