"""GPU: fp32 MFMA GEMMs vs a float64 torch reference (error bound ~1e-6 * sum|a*b|)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref_close(out, ref, absprod, rtol=2e-6):
    err = (out.double() - ref).abs()
    bound = rtol * absprod + 1e-30
    assert bool((err <= bound).all()), float((err / bound).max())


@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (7, 5, 3), (128, 128, 16), (300, 128, 132), (1000, 384, 256),
                                   (257, 512, 384), (4096, 64, 656), (33, 130, 19)])
@pytest.mark.parametrize("transB", [0, 1])
def test_gemm(M, N, K, transB):
    from marlsat import _lib

    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K)
    A = torch.randn(M, K, device="cuda", generator=g)
    B = torch.randn((N, K) if transB else (K, N), device="cuda", generator=g)
    bias = torch.randn(N, device="cuda", generator=g)
    C = torch.randn(M, N, device="cuda", generator=g)
    C0 = C.clone()
    Bop = B.double().t() if transB else B.double()
    for acc in (0, 1):
        C.copy_(C0)
        _lib.check(_lib.lib.msat_gemm(A.data_ptr(), K, B.data_ptr(), B.shape[1], transB, C.data_ptr(), N,
                                      bias.data_ptr(), M, N, K, acc, _lib.stream_ptr()), "gemm")
        ref = A.double() @ Bop + bias.double() + (C0.double() if acc else 0)
        absprod = A.double().abs() @ Bop.abs() + bias.double().abs() + (C0.double().abs() if acc else 0)
        _ref_close(C, ref, absprod)


def test_gemm_strided_column_slices():
    """Write into / read from column slices of wider buffers (the [m_pos | m_neg] concat pattern)."""
    from marlsat import _lib

    M, K, N = 500, 128, 128
    X = torch.randn(M, 2 * K + 4, device="cuda")
    W = torch.randn(K, N, device="cuda")
    Y = torch.zeros(M, 3 * N, device="cuda")
    _lib.check(_lib.lib.msat_gemm(X[:, K:].data_ptr(), 2 * K + 4, W.data_ptr(), N, 0, Y[:, N:].data_ptr(), 3 * N,
                                  None, M, N, K, 0, _lib.stream_ptr()), "gemm")
    ref = X[:, K:2 * K].double() @ W.double()
    _ref_close(Y[:, N:2 * N], ref, X[:, K:2 * K].double().abs() @ W.double().abs())
    assert float(Y[:, :N].abs().max()) == 0 and float(Y[:, 2 * N:].abs().max()) == 0


@pytest.mark.parametrize("M,K,N", [(1, 1, 1), (100, 3, 128), (5000, 256, 384), (70000, 128, 128), (999, 133, 65)])
def test_gemm_wgrad(M, K, N):
    from marlsat import _lib

    A = torch.randn(M, K, device="cuda")
    G = torch.randn(M, N, device="cuda")
    W = torch.randn(K, N, device="cuda")
    W0 = W.clone()
    ws = torch.empty(int(_lib.lib.msat_gemm_wgrad_workspace_bytes(M, K, N)) // 4 + 1, device="cuda")
    for acc in (0, 1):
        W.copy_(W0)
        _lib.check(_lib.lib.msat_gemm_wgrad(A.data_ptr(), K, G.data_ptr(), N, W.data_ptr(), N, M, K, N, acc,
                                            ws.data_ptr(), _lib.stream_ptr()), "wgrad")
        ref = A.double().t() @ G.double() + (W0.double() if acc else 0)
        absprod = A.double().abs().t() @ G.double().abs() + (W0.double().abs() if acc else 0)
        _ref_close(W, ref, absprod, rtol=4e-6)
        W1 = W.clone()
        _lib.check(_lib.lib.msat_gemm_wgrad(A.data_ptr(), K, G.data_ptr(), N, W.data_ptr(), N, M, K, N, 0,
                                            ws.data_ptr(), _lib.stream_ptr()), "wgrad")
        if not acc:
            assert torch.equal(W, W1)  # bitwise reproducible


@pytest.mark.parametrize("M,N,K,transB", [(1, 4, 32, 0), (130, 132, 64, 0), (1000, 384, 256, 0), (257, 128, 384, 1),
                                          (700, 260, 128, 1), (129, 256, 96, 0), (3, 128, 32, 1), (77, 130, 36, 0),
                                          (65, 6, 40, 1)])
def test_gemm_fast_path_shapes(M, N, K, transB):
    """K % 32 == 0 shapes take the LDS-DMA kernel (tails in M and N: clamped reads, masked stores); the
    last two (K % 32 != 0, N % 4 != 0) the register-staged kernel."""
    from marlsat import _lib

    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + 7 * K)
    A = torch.randn(M, K, device="cuda", generator=g)
    B = torch.randn((N, K) if transB else (K, N), device="cuda", generator=g)
    bias = torch.randn(N, device="cuda", generator=g)
    C0 = torch.randn(M, N, device="cuda", generator=g)
    Bop = B.double().t() if transB else B.double()
    for acc in (0, 1):
        C = C0.clone()
        _lib.check(_lib.lib.msat_gemm(A.data_ptr(), K, B.data_ptr(), B.shape[1], transB, C.data_ptr(), N,
                                      bias.data_ptr(), M, N, K, acc, _lib.stream_ptr()), "gemm")
        ref = A.double() @ Bop + bias.double() + (C0.double() if acc else 0)
        absprod = A.double().abs() @ Bop.abs() + bias.double().abs() + (C0.double().abs() if acc else 0)
        _ref_close(C, ref, absprod)


# fp32 MFMA tiles (MARLSAT_PRECISION=fp32) / bf16x3 (whole-row for N <= 384, 128 x 128 tiles above)
@pytest.mark.parametrize("path", ["fp32", "x3"])
@pytest.mark.parametrize("M,K,N", [(1, 4, 4), (33, 128, 384), (5000, 132, 384), (70001, 128, 128), (100, 256, 8),
                                   (407001, 128, 384), (9999, 256, 260), (17, 16, 4), (1000, 12, 36), (3000, 300, 384),
                                   (2049, 256, 512)])
def test_wgrad_fast_path_shapes(M, K, N, path, c_precision):
    """Row tails (M % 32 != 0, splits of uneven length) go through zero-filled slabs; the bf16x3
    kernels (transposed LDS reads) are held to the same fp32 bound as the fp32 MFMA kernels."""
    from marlsat import _lib

    c_precision("fp32" if path == "fp32" else "fp16x2")
    g = torch.Generator(device="cuda").manual_seed(M + K + N)
    A = torch.randn(M, K, device="cuda", generator=g)
    G = torch.randn(M, N, device="cuda", generator=g)
    W0 = torch.randn(K, N, device="cuda", generator=g)
    ws = torch.empty(int(_lib.lib.msat_gemm_wgrad_workspace_bytes(M, K, N)) // 4 + 1, device="cuda")
    for acc in (0, 1):
        W = W0.clone()
        _lib.check(_lib.lib.msat_gemm_wgrad(A.data_ptr(), K, G.data_ptr(), N, W.data_ptr(), N, M, K, N, acc,
                                            ws.data_ptr(), _lib.stream_ptr()), "wgrad")
        ref = A.double().t() @ G.double() + (W0.double() if acc else 0)
        absprod = A.double().abs().t() @ G.double().abs() + (W0.double().abs() if acc else 0)
        _ref_close(W, ref, absprod)


@pytest.mark.parametrize("path", ["x3", "fp32"])
@pytest.mark.parametrize("M,K,N,rot,ldg", [(5000, 128, 384, 256, 512), (70001, 256, 384, 256, 512), (999, 128, 128, 32, 128),
                                           (300, 256, 384, 128, 384), (5000, 128, 512, 256, 512),
                                           (700001, 64, 192, 128, 192)])
def test_wgrad_rot(M, K, N, rot, ldg, path, c_precision):
    """msat_gemm_wgrad_rot: W[:, (n + rot) % N] (+)= (A^T G)[:, n] (the packed GRU backward rows), on the
    whole-row kernel's rotated store (N <= 384) and on the two-range fallback (bf16x3 tiles for N = 512, or
    fp32 MFMA tiles with MARLSAT_PRECISION=fp32); G read from a wider row (ld > N).  The H = 64, 700 K-row case: the fallback's
    128-column sub-product takes more row splits than the full width, and the workspace
    (msat_gemm_wgrad_workspace_bytes) must hold them."""
    from marlsat import _lib

    if path == "fp32" and M < 700001:
        pytest.skip("the fp32 fallback is covered by the large-M case")
    c_precision("fp32" if path == "fp32" else "fp16x2")
    g = torch.Generator(device="cuda").manual_seed(M + K + N + rot)
    A = torch.randn(M, K, device="cuda", generator=g)
    Gw = torch.randn(M, ldg, device="cuda", generator=g)
    G = Gw[:, :N]
    W0 = torch.randn(K, N, device="cuda", generator=g)
    nws = int(_lib.lib.msat_gemm_wgrad_workspace_bytes(M, K, N)) // 4 + 1
    ws = torch.full((nws + (1 << 20),), 7.0, device="cuda")  # + a canary tail that must stay untouched
    for acc in (0, 1):
        W = W0.clone()
        _lib.check(_lib.lib.msat_gemm_wgrad_rot(A.data_ptr(), K, Gw.data_ptr(), ldg, W.data_ptr(), N, M, K, N, rot, acc,
                                                ws.data_ptr(), _lib.stream_ptr()), "wgrad_rot")
        ref = torch.roll(A.double().t() @ G.double(), rot, dims=1) + (W0.double() if acc else 0)
        absprod = torch.roll(A.double().abs().t() @ G.double().abs(), rot, dims=1) + (W0.double().abs() if acc else 0)
        _ref_close(W, ref, absprod)
        assert bool((ws[nws:] == 7.0).all()), "wgrad_rot wrote past its workspace"


def row_exp(G: torch.Tensor) -> torch.Tensor:
    """The fp16x2 row scale exponent (split3.h f16x2_row_exp): max|row| * 2^e in [2^14, 2^15)."""
    m = G.abs().amax(dim=1)
    e = 15 - torch.frexp(m)[1]
    return torch.where(m == 0, torch.full_like(e, 0x3FFF), e).to(torch.int32)


@pytest.mark.parametrize("M,K,N,rot,ldg,amp", [(5000, 128, 384, 256, 512, 0), (70001, 256, 384, 256, 512, 0),
                                               (999, 128, 128, 32, 128, 0), (300, 256, 384, 128, 384, 0),
                                               (407001, 128, 384, 0, 512, 0), (20000, 128, 384, 0, 384, 1),
                                               (3000, 16, 260, 4, 260, 0), (17, 16, 4, 0, 4, 0)])
def test_wgrad_h2(M, K, N, rot, ldg, amp):
    """fp16x2 whole-row weight gradient: rows of G spread over 10^-30 .. 10^2 (and all-zero rows), scaled
    per split by the row exponents; amp = 1 puts |a| >= 2^15 into one split's A rows, which the bf16x3
    fixup launch recomputes.  Held to the fp32 bound against fp64 (max err / sum|a g| printed)."""
    from marlsat import _lib

    g = torch.Generator(device="cuda").manual_seed(M + K + N + rot + amp)
    A = torch.randn(M, K, device="cuda", generator=g)
    if amp:
        A[M // 3: M // 3 + 5] *= 1e6
    Gw = torch.randn(M, ldg, device="cuda", generator=g)
    Gw *= torch.pow(10.0, torch.empty(M, 1, device="cuda").uniform_(-30, 2, generator=g))
    Gw[::7] = 0
    G = Gw[:, :N]
    rexp = row_exp(Gw)
    W0 = torch.randn(K, N, device="cuda", generator=g)
    ws = torch.empty(int(_lib.lib.msat_gemm_wgrad_workspace_bytes(M, K, N)) // 4 + 1, device="cuda")
    for acc in (0, 1):
        W = W0.clone()
        _lib.check(_lib.lib.msat_gemm_wgrad_h2(A.data_ptr(), K, Gw.data_ptr(), ldg, rexp.data_ptr(), W.data_ptr(), N, M,
                                               K, N, rot, acc, ws.data_ptr(), _lib.stream_ptr()), "wgrad_h2")
        ref = torch.roll(A.double().t() @ G.double(), rot, dims=1) + (W0.double() if acc else 0)
        absprod = torch.roll(A.double().abs().t() @ G.double().abs(), rot, dims=1) + (W0.double().abs() if acc else 0)
        _ref_close(W, ref, absprod, rtol=4e-6)
        W1 = W.clone()
        if not acc:
            _lib.check(_lib.lib.msat_gemm_wgrad_h2(A.data_ptr(), K, Gw.data_ptr(), ldg, rexp.data_ptr(), W.data_ptr(),
                                                   N, M, K, N, rot, 0, ws.data_ptr(), _lib.stream_ptr()), "wgrad_h2")
            assert torch.equal(W, W1)  # bitwise reproducible


@pytest.mark.parametrize("M,N,K,rot,lda,wbig,acc", [(1, 128, 384, 256, 512, 0, 0), (130, 128, 384, 0, 512, 0, 1),
                                                     (70001, 256, 384, 256, 512, 0, 0), (4999, 128, 384, 0, 384, 0, 1),
                                                     (3000, 130, 96, 32, 100, 0, 1), (257, 128, 384, 256, 512, 1, 1)])
def test_gemm_h2(M, N, K, rot, lda, wbig, acc):
    """fp16x2 data gradient C (+)= A @ W^T with per-row scale exponents: rows of A spread over 10^-30 .. 10^2
    and all-zero rows; W's gate blocks rotated as in the packed backward (planes of W[:, (c + rot) % K]);
    wbig = 1 puts a weight >= 32 in W (fp16 overflow at 2^10 scale), which runs the bf16x3 body."""
    from marlsat import _lib

    g = torch.Generator(device="cuda").manual_seed(M + N + K + rot + wbig)
    Aw = torch.randn(M, lda, device="cuda", generator=g)
    Aw *= torch.pow(10.0, torch.empty(M, 1, device="cuda").uniform_(-30, 2, generator=g))
    Aw[::5] = 0
    A = Aw[:, :K]
    rexp = row_exp(Aw)
    W = torch.randn(N, K, device="cuda", generator=g) * 0.1
    if wbig:
        W[3, 7] = 40.0
    C0 = torch.randn(M, N, device="cuda", generator=g)
    p2 = torch.empty(2 * N * K + 8, dtype=torch.int16, device="cuda")
    p3 = torch.empty(3 * N * K + 8, dtype=torch.int16, device="cuda")
    bad = torch.empty(1, dtype=torch.int32, device="cuda")
    s = _lib.stream_ptr()
    _lib.check(_lib.lib.msat_split_f16x2_rot(W.data_ptr(), N, K, K, rot, p2.data_ptr(), bad.data_ptr(), s), "split")
    _lib.check(_lib.lib.msat_split_bf16x3_rot(W.data_ptr(), N, K, K, rot, p3.data_ptr(), s), "split3")
    assert int(bad) == wbig
    C = C0.clone()
    _lib.check(_lib.lib.msat_gemm_h2(Aw.data_ptr(), lda, rexp.data_ptr(), p2.data_ptr(), p3.data_ptr(), bad.data_ptr(),
                                     C.data_ptr(), N, None, M, N, K, acc, s), "gemm_h2")
    Wr = torch.roll(W.double(), -rot, dims=1)  # planes hold W[:, (c + rot) % K]
    ref = A.double() @ Wr.t() + (C0.double() if acc else 0)
    absprod = A.double().abs() @ Wr.abs().t() + (C0.double().abs() if acc else 0)
    _ref_close(C, ref, absprod)


@pytest.mark.parametrize("M,K,N,lda,aoff,ldw", [(1, 1, 4, 1, 0, 4), (1000, 3, 384, 4, 1, 384), (300001, 4, 384, 8, 4, 384),
                                                (77777, 8, 260, 8, 0, 264), (5000, 5, 128, 7, 2, 132),
                                                (64, 2, 768, 2, 0, 768)])
def test_wgrad_skinny(M, K, N, lda, aoff, ldw):
    """K <= 8 weight gradients (input features, degree columns) take the streaming reduction:
    unaligned / strided A rows, strided W, accumulate, bitwise repeatable."""
    from marlsat import _lib

    g = torch.Generator(device="cuda").manual_seed(M + 13 * K + N)
    abuf = torch.randn(M * lda + aoff + 8, device="cuda", generator=g)
    A = abuf[aoff:aoff + M * lda].view(M, lda)
    G = torch.randn(M, N, device="cuda", generator=g)
    W0 = torch.randn(K, ldw, device="cuda", generator=g)
    ws = torch.empty(int(_lib.lib.msat_gemm_wgrad_workspace_bytes(M, K, N)) // 4 + 4, device="cuda")
    for acc in (0, 1):
        outs = []
        for _ in range(2):
            W = W0.clone()
            _lib.check(_lib.lib.msat_gemm_wgrad(A.data_ptr(), lda, G.data_ptr(), N, W.data_ptr(), ldw, M, K, N, acc,
                                                ws.data_ptr(), _lib.stream_ptr()), "wgrad")
            outs.append(W)
        assert torch.equal(outs[0], outs[1])
        Ad = A[:, :K].double()
        ref = Ad.t() @ G.double() + (W0[:, :N].double() if acc else 0)
        absprod = Ad.abs().t() @ G.double().abs() + (W0[:, :N].double().abs() if acc else 0)
        _ref_close(outs[0][:, :N], ref, absprod)
        assert torch.equal(outs[0][:, N:], W0[:, N:])


@pytest.mark.parametrize("M,N,ld,off", [(1, 4, 4, 0), (221000, 128, 256, 128), (5000, 384, 384, 0), (777, 7, 9, 1),
                                        (0, 8, 8, 0), (100, 130, 132, 2)])
def test_colsum_deterministic(M, N, ld, off):
    """msat_colsum (bias gradients): float4 path when rows / output are 16-byte addressable, scalar
    path otherwise; fixed reduction order -> identical results on repeat."""
    from marlsat import _lib

    g = torch.Generator(device="cuda").manual_seed(M + N)
    buf = torch.randn(max(M, 1) * ld + off + 8, device="cuda", generator=g)
    G = buf[off:off + M * ld].view(M, ld) if M else buf[:0].view(0, ld)
    oo = off % 4  # output offset: 0 keeps it 16-byte aligned
    out0 = torch.randn(N + 8, device="cuda", generator=g)
    ws = torch.empty(int(_lib.lib.msat_colsum_workspace_floats(M, N)) + 4, device="cuda")
    res = []
    for _ in range(2):
        out = out0.clone()
        _lib.check(_lib.lib.msat_colsum(G.data_ptr(), ld, M, N, out.data_ptr() + 4 * oo, 1, ws.data_ptr(),
                                        _lib.stream_ptr()), "colsum")
        res.append(out)
    assert torch.equal(res[0], res[1])
    ref = out0.double().clone()
    if M:
        ref[oo:oo + N] += G[:, :N].double().sum(0)
    err = (res[0].double() - ref).abs()
    bound = 2e-6 * (G[:, :N].double().abs().sum(0) if M else torch.zeros(N, dtype=torch.float64, device="cuda"))
    assert bool((err[oo:oo + N] <= bound + 1e-6).all())
    assert torch.equal(res[0][:oo], out0[:oo]) and torch.equal(res[0][oo + N:], out0[oo + N:])


@pytest.mark.parametrize("M,N,K,lda", [(1, 4, 16, 16), (130, 132, 64, 64), (1000, 384, 384, 384), (5000, 128, 384, 384),
                                       (257, 256, 128, 128), (3, 7, 32, 32), (77, 100, 48, 52), (5000, 128, 384, 512),
                                       (1001, 256, 384, 384), (77, 100, 64, 68)])
def test_gemm_x3_fp32_accuracy(M, N, K, lda):
    """bf16x3 split GEMM: C = A @ W^T (+ bias, + C) at fp32 accuracy (same bound as the f32 MFMA
    kernels: 2e-6 of sum |a b|), including values spanning many binades and strided A rows.  K % 32 == 0
    takes the register-A 16x16x32 kernel, K % 32 == 16 the LDS-staged one."""
    from marlsat import _lib

    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    A = torch.randn(M, lda, device="cuda", generator=g) * torch.exp2(torch.randint(-6, 7, (M, lda), device="cuda",
                                                                                    generator=g).float())
    W = torch.randn(N, K, device="cuda", generator=g)
    bias = torch.randn(N, device="cuda", generator=g)
    C0 = torch.randn(M, N, device="cuda", generator=g)
    planes = torch.empty(3 * N * K + 8, dtype=torch.int16, device="cuda")
    s = _lib.stream_ptr()
    _lib.check(_lib.lib.msat_split_bf16x3(W.data_ptr(), N, K, K, planes.data_ptr(), s), "split")
    hi, mid, lo = (planes[i * N * K:(i + 1) * N * K].view(torch.bfloat16).float().view(N, K) for i in range(3))
    assert float(((hi.double() + mid.double() + lo.double()) - W.double()).abs().max()) <= \
        2.0 ** -24 * float(W.abs().max())
    Ak = A[:, :K].double()
    for acc in (0, 1):
        C = C0.clone()
        _lib.check(_lib.lib.msat_gemm_x3(A.data_ptr(), lda, planes.data_ptr(), C.data_ptr(), N, bias.data_ptr(), M, N,
                                         K, acc, s), "gemm_x3")
        ref = Ak @ W.double().t() + bias.double() + (C0.double() if acc else 0)
        absprod = Ak.abs() @ W.double().abs().t() + bias.double().abs() + (C0.double().abs() if acc else 0)
        _ref_close(C, ref, absprod)


@pytest.mark.parametrize("M,K1,wbig", [(1, 128, None), (4999, 128, None), (70001, 256, None), (385, 256, "Wh"),
                                       (385, 128, "F"), (4999, 256, "both")])
def test_dual_launches_match_fp64(M, K1, wbig):
    """A GRU cell's two data gradients (msat_gemm_h2_dual) and two weight gradients (msat_gemm_wgrad_h2_dual)
    from one packed buffer D = [dan | dar | daz | dan r] (ld 4H): dh (+)= D[:, H:] @ Wh^T, dx = D[:, :3H] @ F^T,
    dWh (+)= h^T D[:, H:], dF (+)= x^T D[:, :3H] rotated by 2H -- each against fp64 at the fp32 bound.
    wbig: one weight of Wh / F / both at 48 (2^10 * 48 is past fp16's range): the weight split flags it and the
    dual data gradient runs its bf16x3 body (the 12-wave, three-plane form of the 384-row workgroups) for that
    product; M = 385 leaves a one-row last block."""
    from marlsat import _lib

    H = 128
    g = torch.Generator(device="cuda").manual_seed(M + K1)
    D = torch.randn(M, 4 * H, device="cuda", generator=g)
    D *= torch.pow(10.0, torch.empty(M, 1, device="cuda").uniform_(-12, 1, generator=g))
    rexp = row_exp(D)
    Wh = torch.randn(H, 3 * H, device="cuda", generator=g) * 0.1   # dh rows N0 = H, K = 3H
    F = torch.randn(K1, 3 * H, device="cuda", generator=g) * 0.1   # dx rows N1 = K1
    if wbig in ("Wh", "both"):
        Wh[3, 7] = 48.0
    if wbig in ("F", "both"):
        F[K1 - 1, 5] = -48.0
    s = _lib.stream_ptr()
    planes = []
    for Wm in (Wh, F):
        n, k = Wm.shape
        p2 = torch.empty(2 * n * k + 8, dtype=torch.int16, device="cuda")
        p3 = torch.empty(3 * n * k + 8, dtype=torch.int16, device="cuda")
        bad = torch.empty(1, dtype=torch.int32, device="cuda")
        rot = 0 if Wm is Wh else 2 * H
        _lib.check(_lib.lib.msat_split_f16x2_rot(Wm.data_ptr(), n, k, k, rot, p2.data_ptr(), bad.data_ptr(), s), "s2")
        _lib.check(_lib.lib.msat_split_bf16x3_rot(Wm.data_ptr(), n, k, k, rot, p3.data_ptr(), s), "s3")
        planes.append((p2, p3, bad))
        # the split flags exactly the overflowing weight matrices
        assert int(bad.item()) == (1 if wbig == "both" or (wbig == "Wh") == (Wm is Wh) and wbig else 0), wbig
    C0 = torch.randn(M, H, device="cuda", generator=g)
    dh = C0.clone()
    dx = torch.empty(M, K1, device="cuda")
    dgh, dgi = D[:, H:], D[:, :3 * H]
    _lib.check(_lib.lib.msat_gemm_h2_dual(
        dgh.data_ptr(), 4 * H, planes[0][0].data_ptr(), planes[0][1].data_ptr(), planes[0][2].data_ptr(), dh.data_ptr(),
        H, H, 1, dgi.data_ptr(), 4 * H, planes[1][0].data_ptr(), planes[1][1].data_ptr(), planes[1][2].data_ptr(),
        dx.data_ptr(), K1, K1, 0, rexp.data_ptr(), M, 3 * H, s), "dual dgrad")
    Fr = torch.roll(F.double(), -2 * H, dims=1)
    _ref_close(dh, dgh.double() @ Wh.double().t() + C0.double(),
               dgh.double().abs() @ Wh.double().abs().t() + C0.double().abs())
    _ref_close(dx, dgi.double() @ Fr.t(), dgi.double().abs() @ Fr.abs().t())
    hx = torch.randn(M, H, device="cuda", generator=g)
    xx = torch.randn(M, K1, device="cuda", generator=g)
    W0 = torch.randn(H, 3 * H, device="cuda", generator=g)
    W1 = torch.randn(K1, 3 * H, device="cuda", generator=g)
    gW0, gW1 = W0.clone(), W1.clone()
    ws = torch.empty(int(_lib.lib.msat_gemm_wgrad_dual_workspace_bytes(M, H, 3 * H, K1, 3 * H)) // 4 + 1, device="cuda")
    _lib.check(_lib.lib.msat_gemm_wgrad_h2_dual(
        hx.data_ptr(), H, dgh.data_ptr(), 4 * H, gW0.data_ptr(), 3 * H, H, 3 * H, 0,
        xx.data_ptr(), K1, dgi.data_ptr(), 4 * H, gW1.data_ptr(), 3 * H, K1, 3 * H, 2 * H,
        rexp.data_ptr(), M, 1, ws.data_ptr(), s), "dual wgrad")
    _ref_close(gW0, hx.double().t() @ dgh.double() + W0.double(),
               hx.double().abs().t() @ dgh.double().abs() + W0.double().abs(), rtol=4e-6)
    _ref_close(gW1, torch.roll(xx.double().t() @ dgi.double(), 2 * H, dims=1) + W1.double(),
               torch.roll(xx.double().abs().t() @ dgi.double().abs(), 2 * H, dims=1) + W1.double().abs(), rtol=4e-6)
