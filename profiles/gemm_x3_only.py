"""bf16x3 data-gradient GEMM (msat_gemm_x3, C = A @ W^T) on the uf50 training shapes, HIP-event timed.
usage: gemm_x3_only.py [reps]"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import torch
from marlsat import _lib

L = _lib.lib
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
Nv, Nc, H = 407000, 1036000, 128
s = _lib.stream_ptr()
for M, N, K, what in [(Nv, H, 3 * H, "var dh"), (Nc, H, 3 * H, "clause dh"), (Nc, 2 * H, 3 * H, "clause dGIN")]:
    A = torch.randn(M, K, device="cuda"); B = torch.randn(N, K, device="cuda"); C = torch.randn(M, N, device="cuda")
    planes = torch.empty(3 * N * K, dtype=torch.int16, device="cuda")
    L.msat_split_bf16x3(B.data_ptr(), N, K, K, planes.data_ptr(), s)
    acc = int(os.environ.get("GEMM_ACC", "0"))  # 1: C += A @ W^T (the backward's accumulating products)
    f = lambda: L.msat_gemm_x3(A.data_ptr(), K, planes.data_ptr(), C.data_ptr(), N, 0, M, N, K, acc, s)
    f(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        f()
    b.record(); torch.cuda.synchronize()
    us = a.elapsed_time(b) / reps * 1e3
    print(json.dumps({"what": what, "M": M, "N": N, "K": K, "us": round(us, 1),
                      "tflops": round(2 * M * N * K / us / 1e6, 1)}))
