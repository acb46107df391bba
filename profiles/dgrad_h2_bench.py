"""Data-gradient kernels on the training shapes, HIP-event timed: bf16x3 register-A (gemm_x3r16_kernel,
msat_gemm_x3) against fp16x2 (gemm_h2r16_kernel, msat_gemm_h2) with the packed rows' scale exponents.
A = packed backward rows (ld 4H), as in gnn.py.  usage: dgrad_h2_bench.py [reps]"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import torch
from marlsat import _lib

L = _lib.lib
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
Nv, Nc, H = 407000, 1036000, 128
s = _lib.stream_ptr()
for M, N, what, acc in [(Nv, H, "var dh", 1), (Nv, H, "var dNV", 0), (Nc, H, "clause dh", 1), (Nc, 2 * H, "clause dGIN", 0)]:
    K = 3 * H
    D = torch.randn(M, 4 * H, device="cuda")
    m = D.abs().amax(dim=1)
    rexp = torch.where(m == 0, torch.full_like(m, 0x3FFF, dtype=torch.int32), 15 - torch.frexp(m)[1]).to(torch.int32)
    W = torch.randn(N, K, device="cuda") * 0.05
    C = torch.randn(M, N, device="cuda")
    p2 = torch.empty(2 * N * K + 8, dtype=torch.int16, device="cuda")
    p3 = torch.empty(3 * N * K + 8, dtype=torch.int16, device="cuda")
    bad = torch.empty(1, dtype=torch.int32, device="cuda")
    L.msat_split_f16x2_rot(W.data_ptr(), N, K, K, 0, p2.data_ptr(), bad.data_ptr(), s)
    L.msat_split_bf16x3_rot(W.data_ptr(), N, K, K, 0, p3.data_ptr(), s)
    fx = lambda: L.msat_gemm_x3(D.data_ptr(), 4 * H, p3.data_ptr(), C.data_ptr(), N, None, M, N, K, acc, s)
    fh = lambda: L.msat_gemm_h2(D.data_ptr(), 4 * H, rexp.data_ptr(), p2.data_ptr(), p3.data_ptr(), bad.data_ptr(),
                                C.data_ptr(), N, None, M, N, K, acc, s)
    for name, f in (("x3r16", fx), ("h2r16", fh)):
        f(); torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            f()
        b.record(); torch.cuda.synchronize()
        us = a.elapsed_time(b) / reps * 1e3
        print(json.dumps({"what": what, "M": M, "N": N, "K": K, "acc": acc, "kernel": name, "us": round(us, 1),
                          "tflops_fp32_equiv": round(2 * M * N * K / us / 1e6, 1),
                          "hbm_GBps": round(M * (K + N * (1 + acc)) * 4 / us / 1e3, 1)}), flush=True)
    del D, C
    torch.cuda.empty_cache()
