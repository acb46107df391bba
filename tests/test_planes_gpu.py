"""GPU: the GRU backward's packed rows as fp16x2 planes (round 5) and the two dual products that consume them.

msat_gru_ln_bwd_g4fe with flags bit 3 stores each packed row [dan | dar | daz | dan r] as [hi | lo] fp16 planes at
its row exponent instead of fp32.  Pinned here:
  * the planes are BITWISE the host split of the fp32 rows the same launch writes without bit 3 (every other
    output -- rexp, dh_prev, the LN / bias / feature gradients -- bitwise unchanged), for the scalar (clause,
    nfeat 2) and vector (var, nfeat 6) bodies, with all-zero rows;
  * msat_gemm_h2_dual_planes is BITWISE msat_gemm_h2_dual on the fp32 rows (the planes are the split it makes),
    and its bf16x3 body (an overflowing weight split) stays inside the fp32 bound;
  * msat_gemm_wgrad_h2_dual_planes (G by LDS-DMA, the split-wide scale moved to A) against fp64 at the bound of
    the fp32-row form (rtol 4e-6 of sum |a g|), with rows spread over 10^-12 .. 10^1, zero rows, a split whose A
    rows pass 2^15 (the bf16x3 fixup rebuilds G from the planes), one-row and ragged last slabs, and 2.2 M rows
    (24 K rows per split, 1.5 K slabs through the four-slot DMA rings) -- and bitwise repeatable.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

H = 128
KZERO = 0x3FFF


def _ref_close(out, ref, absprod, rtol=2e-6):
    err = (out.double() - ref).abs()
    bound = rtol * absprod + 1e-30
    assert bool((err <= bound).all()), float((err / bound).max())


def row_exp(G: torch.Tensor) -> torch.Tensor:
    m = G.abs().amax(dim=1)
    e = 15 - torch.frexp(m)[1]
    return torch.where(m == 0, torch.full_like(e, KZERO), e).to(torch.int32)


def pow2(e: torch.Tensor) -> torch.Tensor:
    """2^e exactly (int32 e in [-126, 127]) from its bits (torch.pow / exp2 on the device need not be exact)."""
    return ((e.to(torch.int32) + 127) << 23).view(torch.float32)


def host_planes(D: torch.Tensor, rexp: torch.Tensor) -> torch.Tensor:
    """(M, 2 W) fp16: [hi | lo] of each row of D at its exponent (kExpZero -> 0), the split of gnn_kernels.hip
    put_h2: hi = fp16(x 2^e), lo = fp16(x 2^e - hi); x 2^e in two exact power-of-two steps."""
    es = torch.where(rexp == KZERO, torch.zeros_like(rexp), rexp).unsqueeze(1)
    e1 = torch.div(es, 2, rounding_mode="floor")
    x = D * pow2(e1) * pow2(es - e1)
    hi = x.half()
    return torch.cat([hi, (x - hi.float()).half()], dim=1).contiguous()


@pytest.mark.parametrize("nfeat,R", [(2, 20011), (6, 20011), (2, 1), (6, 3)])
def test_gru_bwd_planes_are_the_split_of_the_fp32_rows(nfeat, R):
    from marlsat import _lib

    L, dev = _lib.lib, "cuda"
    g = torch.Generator(device=dev).manual_seed(R + nfeat)
    dy = torch.randn(R, H, device=dev, generator=g)
    dy[::9] = 0  # all-zero packed rows (kExpZero)
    dy *= torch.pow(10.0, torch.empty(R, 1, device=dev).uniform_(-8, 1, generator=g))
    g4 = torch.randn(R, 4 * H, device=dev, generator=g)
    hp = torch.randn(R, H, device=dev, generator=g)
    sc = torch.randn(H, device=dev, generator=g)
    ldf = 8 if nfeat == 6 else 4
    feat = torch.randn(R, ldf, device=dev, generator=g)
    part = torch.empty(int(L.msat_gru_ln_bwd_partial_floats(R, H)), device=dev)
    s = _lib.stream_ptr()
    seeds = [torch.randn(2 * H, device=dev, generator=g), torch.randn(3 * H, device=dev, generator=g),
             torch.randn(3 * H, device=dev, generator=g), torch.randn(nfeat, 3 * H, device=dev, generator=g)]

    def run(flags):
        D = torch.empty(R, 4 * H, device=dev)
        dh = torch.empty(R, H, device=dev)
        dln, dbi, dbh, dfeat = (t.clone() for t in seeds)
        rexp = torch.empty(R, dtype=torch.int32, device=dev)
        _lib.check(L.msat_gru_ln_bwd_g4fe(dy.data_ptr(), H, g4.data_ptr(), 4 * H, hp.data_ptr(), H, sc.data_ptr(),
                                          D.data_ptr(), 4 * H, D.data_ptr() + 4 * H, 4 * H, dh.data_ptr(), H,
                                          dln.data_ptr(), dln.data_ptr() + 4 * H, dbi.data_ptr(),
                                          dbh.data_ptr() + 4 * 2 * H, feat.data_ptr(), ldf, nfeat, dfeat.data_ptr(),
                                          part.data_ptr(), R, H, flags, rexp.data_ptr(), s), "gru_ln_bwd_g4fe")
        return D, rexp, (dh, dln, dbi, dbh, dfeat)

    D32, rexp32, outs32 = run(7)
    Dp, rexpp, outsp = run(15)
    torch.cuda.synchronize()
    assert torch.equal(rexp32, rexpp)
    for a, b in zip(outs32, outsp):
        assert torch.equal(a, b)
    got = Dp.view(torch.int16).view(R, 8 * H)
    want = host_planes(D32, rexp32).view(torch.int16)
    assert torch.equal(got, want)
    assert bool((rexp32[::9] == KZERO).all())


def _weights(Wm, rot, s, L):
    n, k = Wm.shape
    p2 = torch.empty(2 * n * k + 8, dtype=torch.int16, device="cuda")
    p3 = torch.empty(3 * n * k + 8, dtype=torch.int16, device="cuda")
    bad = torch.empty(1, dtype=torch.int32, device="cuda")
    L.msat_split_f16x2_rot(Wm.data_ptr(), n, k, k, rot, p2.data_ptr(), bad.data_ptr(), s)
    L.msat_split_bf16x3_rot(Wm.data_ptr(), n, k, k, rot, p3.data_ptr(), s)
    return p2, p3, bad


@pytest.mark.parametrize("M,K1,wbig", [(1, 128, None), (385, 256, None), (4999, 128, None), (70001, 256, None),
                                       (385, 256, "Wh"), (4999, 128, "both")])
def test_dual_dgrad_planes_is_bitwise_the_fp32_row_form(M, K1, wbig):
    from marlsat import _lib

    L, s = _lib.lib, _lib.stream_ptr()
    g = torch.Generator(device="cuda").manual_seed(M + K1 + 3)
    D = torch.randn(M, 4 * H, device="cuda", generator=g)
    D *= torch.pow(10.0, torch.empty(M, 1, device="cuda").uniform_(-12, 1, generator=g))
    D[1::7] = 0
    rexp = row_exp(D)
    P = host_planes(D, rexp)
    Wh = torch.randn(H, 3 * H, device="cuda", generator=g) * 0.1
    F = torch.randn(K1, 3 * H, device="cuda", generator=g) * 0.1
    if wbig in ("Wh", "both"):
        Wh[3, 7] = 48.0
    if wbig == "both":
        F[K1 - 1, 5] = -48.0
    w0, w1 = _weights(Wh, 0, s, L), _weights(F, 2 * H, s, L)
    C0 = torch.randn(M, H, device="cuda", generator=g)
    res = []
    for planes in (0, 1):
        dh, dx = C0.clone(), torch.empty(M, K1, device="cuda")
        if planes:
            _lib.check(L.msat_gemm_h2_dual_planes(
                P.data_ptr() + 2 * H, 8 * H, w0[0].data_ptr(), w0[1].data_ptr(), w0[2].data_ptr(), dh.data_ptr(), H,
                H, 1, P.data_ptr(), 8 * H, w1[0].data_ptr(), w1[1].data_ptr(), w1[2].data_ptr(), dx.data_ptr(), K1,
                K1, 0, 4 * H, rexp.data_ptr(), M, 3 * H, s), "dual dgrad planes")
        else:
            _lib.check(L.msat_gemm_h2_dual(
                D.data_ptr() + 4 * H, 4 * H, w0[0].data_ptr(), w0[1].data_ptr(), w0[2].data_ptr(), dh.data_ptr(), H,
                H, 1, D.data_ptr(), 4 * H, w1[0].data_ptr(), w1[1].data_ptr(), w1[2].data_ptr(), dx.data_ptr(), K1,
                K1, 0, rexp.data_ptr(), M, 3 * H, s), "dual dgrad")
        res.append((dh, dx))
    dgh, dgi = D[:, H:], D[:, :3 * H]
    Fr = torch.roll(F.double(), -2 * H, dims=1)
    for dh, dx in res:
        _ref_close(dh, dgh.double() @ Wh.double().t() + C0.double(),
                   dgh.double().abs() @ Wh.double().abs().t() + C0.double().abs())
        _ref_close(dx, dgi.double() @ Fr.t(), dgi.double().abs() @ Fr.abs().t())
    # fp16x2 bodies: the same operands bit for bit; a bf16x3 body rebuilds A from the planes (22 bits), so only
    # the products whose weights fit fp16 are held bitwise
    if wbig in (None,):
        assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    elif wbig == "Wh":
        assert torch.equal(res[0][1], res[1][1])


@pytest.mark.parametrize("M,K1,amp", [(1, 128, 0), (17, 256, 0), (385, 256, 0), (4999, 128, 0), (70001, 256, 0),
                                      (20000, 128, 1), (20000, 256, 2), (2200001, 256, 0), (20000, 256, 3),
                                      (70001, 128, 4)])
def test_dual_wgrad_planes_match_fp64(M, K1, amp):
    from marlsat import _lib

    L, s = _lib.lib, _lib.stream_ptr()
    g = torch.Generator(device="cuda").manual_seed(M + K1 + amp)
    D = torch.randn(M, 4 * H, device="cuda", generator=g)
    D *= torch.pow(10.0, torch.empty(M, 1, device="cuda").uniform_(-12, 1, generator=g))
    D[2::11] = 0
    rexp = row_exp(D)
    P = host_planes(D, rexp)
    hx = torch.randn(M, H, device="cuda", generator=g)
    xx = torch.randn(M, K1, device="cuda", generator=g)
    if amp == 1:  # a' past fp16's range in one split's rows: flagged, recomputed by the bf16x3 fixup from the planes
        hx[M // 3: M // 3 + 5] *= 1e6
    if amp == 2:  # |a| up to ~250: a' = a 2^8 up to fp16's largest finite values, still the fp16x2 path
        xx[M // 2: M // 2 + 7] *= 60.0
    if amp == 3:  # every activation tiny: a' fp16-subnormal in every column -> every workgroup's fixup
        hx *= 1e-6
        xx *= 1e-6
    if amp == 4:  # single collapsed columns (a LayerNorm unit whose scale went to ~0) beside normal ones
        hx[:, 5] *= 1e-7
        xx[:, 9] *= 1e-8
        xx[:, K1 - 1] = 0.0  # an all-zero column needs no fixup (its products are zero)
    W0 = torch.randn(H, 3 * H, device="cuda", generator=g)
    W1 = torch.randn(K1, 3 * H, device="cuda", generator=g)
    if amp in (3, 4):  # nothing to add to: the bar is then the tiny products' own 4e-6 of sum |a g|
        W0.zero_()
        W1.zero_()
    ws = torch.empty(int(L.msat_gemm_wgrad_dual_workspace_bytes(M, H, 3 * H, K1, 3 * H)) // 4 + 1, device="cuda")
    outs = []
    for _ in range(2):
        gW0, gW1 = W0.clone(), W1.clone()
        _lib.check(L.msat_gemm_wgrad_h2_dual_planes(
            hx.data_ptr(), H, P.data_ptr() + 2 * H, 8 * H, gW0.data_ptr(), 3 * H, H, 3 * H, 0,
            xx.data_ptr(), K1, P.data_ptr(), 8 * H, gW1.data_ptr(), 3 * H, K1, 3 * H, 2 * H,
            4 * H, rexp.data_ptr(), M, 1, ws.data_ptr(), s), "dual wgrad planes")
        outs.append((gW0, gW1))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])  # bitwise repeatable
    gW0, gW1 = outs[0]
    dgh, dgi = D[:, H:].double(), D[:, :3 * H].double()
    _ref_close(gW0, hx.double().t() @ dgh + W0.double(), hx.double().abs().t() @ dgh.abs() + W0.double().abs(),
               rtol=4e-6)
    _ref_close(gW1, torch.roll(xx.double().t() @ dgi, 2 * H, dims=1) + W1.double(),
               torch.roll(xx.double().abs().t() @ dgi.abs(), 2 * H, dims=1) + W1.double().abs(), rtol=4e-6)
