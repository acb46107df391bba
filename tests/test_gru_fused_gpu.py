"""GPU: fused GRU cell + LayerNorm (msat_gru_ln_fused_fwd / msat_gru_ln_bwd_g4) vs a float64
torch restatement of flax nn.GRUCell + nn.LayerNorm (learner:68-80).

Inputs are segmented exactly as the encoder calls them: the var cells read
x = [n_v (H, a column slice of a 2H buffer) | x, svf (4)], the clause cell
x = [m_c+ | m_c-] (2H).  Row counts include 0, ragged tails (not a multiple of the
64-row tile) and a size large enough to fill the chip.  Tolerances: h' 1e-5 relative
+ 1e-5 absolute (LayerNorm output is O(1)); pre-activation tape 2e-6 of sum|terms|;
gradients 1e-4 of the tensor's max magnitude."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref_gru_ln(x, h, wi, bi, wh, bh, sc, lb, H):
    gi = x @ wi + bi
    gh = h @ wh + bh
    r = torch.sigmoid(gi[:, :H] + gh[:, :H])
    z = torch.sigmoid(gi[:, H:2 * H] + gh[:, H:2 * H])
    n = torch.tanh(gi[:, 2 * H:] + r * gh[:, 2 * H:])
    hn = (1 - z) * n + z * h
    mean = hn.mean(-1, keepdim=True)
    var = (hn * hn).mean(-1, keepdim=True) - mean * mean
    return (hn - mean) * torch.rsqrt(var + 1e-6) * sc + lb, gi, gh


def _setup(R, H, kind, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    rnd = lambda *s: torch.randn(*s, device="cuda", generator=g)
    if kind == "var":
        NV = rnd(R, 2 * H)
        vf = rnd(R, 4)
        segs = [(NV, H, 2 * H, H), (vf, 0, 4, 4)]  # (tensor, col offset, ld, width)
        x = torch.cat([NV[:, H:], vf], 1)
        Kx = H + 4
    elif kind == "var8":  # fused encoder: [gathered half | x, svf, n+, n-, 0, 0]
        NV = rnd(R, 2 * H)
        vf = rnd(R, 8)
        segs = [(NV, 0, 2 * H, H), (vf, 0, 8, 8)]
        x = torch.cat([NV[:, :H], vf], 1)
        Kx = H + 8
    elif kind == "clause4":  # fused encoder: [gathered (2H) | n+, n-, 0, 0]
        GIN = rnd(R, 2 * H)
        cd = rnd(R, 4)
        segs = [(GIN, 0, 2 * H, 2 * H), (cd, 0, 4, 4)]
        x = torch.cat([GIN, cd], 1)
        Kx = 2 * H + 4
    else:
        GIN = rnd(R, 2 * H)
        segs = [(GIN, 0, 2 * H, 2 * H)]
        x = GIN
        Kx = 2 * H
    h = rnd(R, H)
    wi = rnd(Kx, 3 * H) / Kx ** 0.5
    wh = rnd(H, 3 * H) / H ** 0.5
    bi = rnd(3 * H) * 0.1
    bh = torch.cat([torch.zeros(2 * H, device="cuda"), rnd(H) * 0.1])
    sc = 1 + 0.1 * rnd(H)
    lb = 0.1 * rnd(H)
    return segs, x, h, wi, bi, wh, bh, sc, lb


def _fwd(segs, h, wi, bi, wh, bh, sc, lb, R, H, g4, layout="plain"):
    from marlsat import _lib

    out = torch.empty(R, H, device="cuda")
    args = []
    for t, off, ld, w in segs + [(None, 0, 0, 0)] * (3 - len(segs)):
        args += [t.data_ptr() + 4 * off if t is not None else 0, ld, w]
    if layout == "x3r":  # register-A bf16x3 kernel (16x16x32): transposed planes W^T, K padded to 32
        K = wi.shape[0]
        kxp = (K + 31) // 32 * 32
        pi = torch.empty(3 * 3 * H * kxp + 8, dtype=torch.int16, device="cuda")
        ph = torch.empty(3 * 3 * H * H + 8, dtype=torch.int16, device="cuda")
        s = _lib.stream_ptr()
        _lib.check(_lib.lib.msat_split_bf16x3_t(wi.data_ptr(), K, 3 * H, 3 * H, kxp, pi.data_ptr(), s), "split_t")
        _lib.check(_lib.lib.msat_split_bf16x3_t(wh.data_ptr(), H, 3 * H, 3 * H, H, ph.data_ptr(), s), "split_t")
        _lib.check(_lib.lib.msat_gru_ln_fused_fwd_x3r(*args, h.data_ptr(), H, pi.data_ptr(), kxp, bi.data_ptr(),
                                                      ph.data_ptr(), bh.data_ptr(), sc.data_ptr(), lb.data_ptr(),
                                                      out.data_ptr(), H, g4.data_ptr() if g4 is not None else 0,
                                                      4 * H, R, H, s), "gru_ln_fused_fwd_x3r")
        torch.cuda.synchronize()
        return out
    if layout == "h2r":  # register-A fp16x2 kernel + bf16x3 fixup of out-of-range tiles
        K = wi.shape[0]
        kxp = (K + 31) // 32 * 32
        s = _lib.stream_ptr()
        pi = torch.empty(3 * 3 * H * kxp + 8, dtype=torch.int16, device="cuda")
        ph = torch.empty(3 * 3 * H * H + 8, dtype=torch.int16, device="cuda")
        qi = torch.empty(2 * 3 * H * kxp + 8, dtype=torch.int16, device="cuda")
        qh = torch.empty(2 * 3 * H * H + 8, dtype=torch.int16, device="cuda")
        bad = torch.full((2,), 7, dtype=torch.int32, device="cuda")
        flags = torch.full(((R + 127) // 128 + 1,), 7, dtype=torch.int32, device="cuda")
        _lib.check(_lib.lib.msat_split_bf16x3_t(wi.data_ptr(), K, 3 * H, 3 * H, kxp, pi.data_ptr(), s), "split_t")
        _lib.check(_lib.lib.msat_split_bf16x3_t(wh.data_ptr(), H, 3 * H, 3 * H, H, ph.data_ptr(), s), "split_t")
        _lib.check(_lib.lib.msat_split_f16x2_t(wi.data_ptr(), K, 3 * H, 3 * H, kxp, qi.data_ptr(), bad.data_ptr(), s),
                   "split_f16x2_t")
        _lib.check(_lib.lib.msat_split_f16x2_t(wh.data_ptr(), H, 3 * H, 3 * H, H, qh.data_ptr(), bad.data_ptr() + 4,
                                                s), "split_f16x2_t")
        _lib.check(_lib.lib.msat_gru_ln_fused_fwd_h2r(*args, h.data_ptr(), H, qi.data_ptr(), qh.data_ptr(),
                                                      pi.data_ptr(), ph.data_ptr(), kxp, bi.data_ptr(), bh.data_ptr(),
                                                      sc.data_ptr(), lb.data_ptr(), out.data_ptr(), H,
                                                      g4.data_ptr() if g4 is not None else 0, 4 * H, R, H,
                                                      flags.data_ptr(), bad.data_ptr(), s), "gru_ln_fused_fwd_h2r")
        torch.cuda.synchronize()
        _fwd.last_flags = (flags[:(R + 127) // 128].cpu(), bad.cpu())
        return out
    _lib.check(_lib.lib.msat_gru_ln_fused_fwd(*args, h.data_ptr(), H, wi.data_ptr(), bi.data_ptr(), wh.data_ptr(),
                                              bh.data_ptr(), sc.data_ptr(), lb.data_ptr(), out.data_ptr(), H,
                                              g4.data_ptr() if g4 is not None else 0, 4 * H, R, H,
                                              _lib.stream_ptr()), "gru_ln_fused_fwd")
    return out


def _fwd_cases():
    """(layout, H, R): the fp32 kernel at H 64 / 128 / 256, the register-A bf16x3 and fp16x2 kernels at
    H 128; the 70,000-row case at the production width H = 128 only."""
    widths = {"plain": (64, 128, 256), "x3r": (128,), "h2r": (128,)}
    return [(lay, H, R) for lay, hs in widths.items() for H in hs for R in (0, 1, 77, 1000, 70000)
            if R != 70000 or H == 128]


@pytest.mark.parametrize("layout,H,R", _fwd_cases())
@pytest.mark.parametrize("kind", ["var", "clause", "var8", "clause4"])
def test_fused_forward_matches_reference(R, H, kind, layout):
    segs, x, h, wi, bi, wh, bh, sc, lb = _setup(R, H, kind, seed=R + H)
    g4 = torch.full((R, 4 * H), float("nan"), device="cuda")
    out = _fwd(segs, h, wi, bi, wh, bh, sc, lb, R, H, g4, layout)
    out_nt = _fwd(segs, h, wi, bi, wh, bh, sc, lb, R, H, None, layout)  # inference form (no tape)
    torch.cuda.synchronize()
    assert torch.equal(out, out_nt)
    if R == 0:
        return
    d = lambda t: t.double()
    ref, gi, gh = _ref_gru_ln(d(x), d(h), d(wi), d(bi), d(wh), d(bh), d(sc), d(lb), H)
    err = (out.double() - ref).abs()
    assert bool((err <= 1e-5 * ref.abs() + 1e-5).all()), float(err.max())
    # tape: [r_pre | z_pre | gin | ghn]
    tape_ref = torch.cat([gi[:, :H] + gh[:, :H], gi[:, H:2 * H] + gh[:, H:2 * H], gi[:, 2 * H:], gh[:, 2 * H:]], 1)
    absx = torch.cat([d(x).abs() @ d(wi).abs() + d(bi).abs(), d(h).abs() @ d(wh).abs() + d(bh).abs()], 1)
    ab = torch.cat([absx[:, :H] + absx[:, 3 * H:4 * H], absx[:, H:2 * H] + absx[:, 4 * H:5 * H],
                    absx[:, 2 * H:3 * H], absx[:, 5 * H:]], 1)
    terr = (g4.double() - tape_ref).abs()
    assert bool((terr <= 2e-6 * ab + 1e-30).all()), float((terr / (ab + 1e-30)).max())


@pytest.mark.parametrize("kind", ["var8", "clause4"])
def test_h2r_small_activations_keep_22_bits(kind):
    """fp16x2 keeps 22 significant bits of an activation only while its low half stays in fp16's normal range;
    the kernel scales the activations by 2^7 before the split so that this holds down to |a| ~ 1e-3.  Every
    activation here is ~1e-3 (inputs and h), biases 0: the tape must stay within fp32 accumulation error of
    float64 (<= 5e-7 of sum|terms|).  Split unscaled, each such activation carried an absolute 2^-25, several
    times that bound -- the error that moved the headline train cycle's var-negative n-gate bias gradients by 10x
    fp32's own (profiles/r06/r06s_* holds both builds' numbers)."""
    H, R = 128, 1000
    segs, x, h, wi, bi, wh, bh, sc, lb = _setup(R, H, kind, seed=11)
    for t, _, _, _ in segs:
        t.mul_(1e-3)
    h = h * 1e-3
    x = x * 1e-3
    bi, bh = torch.zeros_like(bi), torch.zeros_like(bh)
    g4 = torch.empty(R, 4 * H, device="cuda")
    out = _fwd(segs, h, wi, bi, wh, bh, sc, lb, R, H, g4, "h2r")
    flags, bad = _fwd.last_flags
    assert int(flags.sum()) == 0 and bad.tolist() == [0, 0]
    d = lambda t: t.double()
    ref, gi, gh = _ref_gru_ln(d(x), d(h), d(wi), d(bi), d(wh), d(bh), d(sc), d(lb), H)
    tape_ref = torch.cat([gi[:, :H] + gh[:, :H], gi[:, H:2 * H] + gh[:, H:2 * H], gi[:, 2 * H:], gh[:, 2 * H:]], 1)
    absx = torch.cat([d(x).abs() @ d(wi).abs(), d(h).abs() @ d(wh).abs()], 1)
    ab = torch.cat([absx[:, :H] + absx[:, 3 * H:4 * H], absx[:, H:2 * H] + absx[:, 4 * H:5 * H],
                    absx[:, 2 * H:3 * H], absx[:, 5 * H:]], 1)
    rel = ((g4.double() - tape_ref).abs() / ab).max().item()
    print(f"small activations ({kind}): tape error / sum|terms| max {rel:.3g}")
    assert rel <= 5e-7, rel
    assert bool(((out.double() - ref).abs() <= 1e-5 * ref.abs() + 1e-5).all())


@pytest.mark.parametrize("big", [4.0e4, 256.0])
@pytest.mark.parametrize("R,bad_tiles", [(1000, (1, 6)), (70000, (0, 300, 546))])
@pytest.mark.parametrize("kind", ["var8", "clause4"])
def test_h2r_out_of_range_tiles_take_the_bf16x3_path(kind, R, bad_tiles, big):
    """fp16x2 range check: activations with |a| >= 256 (2^15 after the kernel's 2^7 pre-scale) in a row flag
    exactly its 128-row tile, which the fixup launch recomputes in bf16x3 (bitwise the x3r kernel's rows
    there), the other tiles keep the fp16x2 result, also where |a| is just inside the range (255 in tile 2 /
    200); weights with |W| >= 32 flag the split and every tile is bf16x3.  70,000 rows: the first tile, one
    in the middle and the last, partial tile (546)."""
    H = 128
    segs, x, h, wi, bi, wh, bh, sc, lb = _setup(R, H, kind, seed=3)
    for i, t in enumerate(bad_tiles):
        segs[0][0][min(R - 1, 128 * t + 2 + 37 * i), 5 + 12 * i] = big * (-1) ** i
    segs[0][0][128 * 2 + 9, 3] = -255.0  # inside the range: tile 2 stays fp16x2
    x = torch.cat([segs[0][0][:, segs[0][1]:segs[0][1] + segs[0][3]], segs[1][0]], 1)
    g4 = torch.empty(R, 4 * H, device="cuda")
    out = _fwd(segs, h, wi, bi, wh, bh, sc, lb, R, H, g4, "h2r")
    flags, bad = _fwd.last_flags
    assert bad.tolist() == [0, 0]
    flagged = set(bad_tiles)
    assert flags.tolist() == [1 if t in flagged else 0 for t in range((R + 127) // 128)]
    g4x = torch.empty(R, 4 * H, device="cuda")
    ox = _fwd(segs, h, wi, bi, wh, bh, sc, lb, R, H, g4x, "x3r")
    for t in sorted(flagged):
        rows = slice(128 * t, min(R, 128 * t + 128))
        assert torch.equal(out[rows], ox[rows]) and torch.equal(g4[rows], g4x[rows])
    d = lambda t: t.double()
    ref, _, _ = _ref_gru_ln(d(x), d(h), d(wi), d(bi), d(wh), d(bh), d(sc), d(lb), H)
    err = (out.double() - ref).abs()
    assert bool((err <= 1e-5 * ref.abs() + 1e-5).all()), float(err.max())
    big = wh * 400.0  # |W| >= 32 somewhere
    out2 = _fwd(segs, h, wi, bi, big, bh, sc, lb, R, H, None, "h2r")
    flags2, bad2 = _fwd.last_flags
    assert bad2.tolist() == [0, 1] and bool((flags2 == 1).all())
    assert torch.equal(out2, _fwd(segs, h, wi, bi, big, bh, sc, lb, R, H, None, "x3r"))


@pytest.mark.parametrize("nfeat", [0, 2, 6])  # msat_gru_ln_bwd_g4f feature-weighted gate sums
@pytest.mark.parametrize("assign", [False, True])  # flags bit 1: dhprev overwritten, never read
@pytest.mark.parametrize("R,H", [(77, 64), (1000, 128), (300, 256)])
def test_g4_backward_matches_autograd(R, H, assign, nfeat):
    from marlsat import _lib

    segs, x, h, wi, bi, wh, bh, sc, lb = _setup(R, H, "var", seed=7 * R + H)
    g4 = torch.empty(R, 4 * H, device="cuda")
    _fwd(segs, h, wi, bi, wh, bh, sc, lb, R, H, g4)
    dy = torch.randn(R, H, device="cuda", generator=torch.Generator(device="cuda").manual_seed(5))
    dGi = torch.empty(R, 3 * H, device="cuda")
    dGh = torch.empty(R, 3 * H, device="cuda")
    dh = torch.full((R, H), float("nan"), device="cuda") if assign else torch.zeros(R, H, device="cuda")
    dln = torch.zeros(2 * H, device="cuda")
    dbi = torch.full((3 * H,), 0.5, device="cuda")  # accumulated into
    dbh = torch.full((3 * H,), 0.5, device="cuda")
    part = torch.empty(int(_lib.lib.msat_gru_ln_bwd_partial_floats(R, H)), device="cuda")
    feat = torch.randn(R, 8, device="cuda", generator=torch.Generator(device="cuda").manual_seed(6))
    dfeat = torch.full((max(nfeat, 1), 3 * H), 0.25, device="cuda")
    _lib.check(_lib.lib.msat_gru_ln_bwd_g4f(dy.data_ptr(), H, g4.data_ptr(), 4 * H, h.data_ptr(), H, sc.data_ptr(),
                                            dGi.data_ptr(), 3 * H, dGh.data_ptr(), 3 * H, dh.data_ptr(), H,
                                            dln.data_ptr(), dln.data_ptr() + 4 * H, dbi.data_ptr(),
                                            dbh.data_ptr() + 4 * 2 * H, feat.data_ptr() if nfeat else 0, 8, nfeat,
                                            dfeat.data_ptr() if nfeat else 0, part.data_ptr(), R, H,
                                            3 if assign else 1, _lib.stream_ptr()), "gru_ln_bwd_g4f")
    torch.cuda.synchronize()
    # autograd through the float64 reference w.r.t. gi, gh (pre-activation gate vectors), h, LN params
    d = lambda t: t.double().detach().requires_grad_(True)
    xd, hd, scd, lbd = d(x), d(h), d(sc), d(lb)
    gi = (xd @ wi.double() + bi.double()).detach().requires_grad_(True)
    gh = (hd @ wh.double() + bh.double()).detach().requires_grad_(True)
    r = torch.sigmoid(gi[:, :H] + gh[:, :H])
    z = torch.sigmoid(gi[:, H:2 * H] + gh[:, H:2 * H])
    n = torch.tanh(gi[:, 2 * H:] + r * gh[:, 2 * H:])
    hn = (1 - z) * n + z * hd
    mean = hn.mean(-1, keepdim=True)
    var = (hn * hn).mean(-1, keepdim=True) - mean * mean
    y = (hn - mean) * torch.rsqrt(var + 1e-6) * scd + lbd
    (y * dy.double()).sum().backward()
    for got, ref, what in ((dGi, gi.grad, "dGi"), (dGh, gh.grad, "dGh"), (dh, hd.grad, "dh"),
                           (dln[:H], scd.grad, "dscale"), (dln[H:], lbd.grad, "dbias"),
                           (dbi - 0.5, gi.grad.sum(0), "dbi"), (dbh[2 * H:] - 0.5, gh.grad[:, 2 * H:].sum(0), "dbh_n")):
        scale = float(ref.abs().max())
        err = float((got.double() - ref).abs().max())
        assert err <= 1e-4 * scale + 1e-6, (what, err, scale)
    assert bool((dbh[:2 * H] == 0.5).all())  # b_hr / b_hz do not exist (flax): untouched
    if nfeat:
        ref = feat[:, :nfeat].double().t() @ gi.grad  # (nfeat, 3H): gates r, z, n
        got = dfeat.double() - 0.25
        scale = float(ref.abs().max())
        assert float((got - ref).abs().max()) <= 1e-4 * scale + 1e-6
