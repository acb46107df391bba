"""fp32 MFMA GEMM / weight-gradient timings on the MAPPO training shapes of the bench
(uf50, micro-batch 1,366: var rows Nv = 407k, clause rows Nc = 1.036M, H = 128), HIP-event
timed; run under rocprofv3 --pmc for per-dispatch counters.  usage: gemm_train_shapes.py [reps]"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import torch
from marlsat import _lib

L = _lib.lib
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
Nv, Nc, H = 407000, 1036000, 128
GEMMS = [(Nv, H, 3 * H, 1, "var dh / dn = dG W^T"), (Nc, H, 3 * H, 1, "clause dh = dGh Wh^T"),
         (Nc, 2 * H, 3 * H, 1, "clause dGIN = dGi F^T")]
WGRADS = [(Nv, H, 3 * H, "var dWh / dF"), (Nc, H, 3 * H, "clause dWh"), (Nc, 2 * H, 3 * H, "clause dF")]


def timeit(fn):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


s = _lib.stream_ptr()
for M, N, K, tb, what in GEMMS:
    A = torch.randn(M, K, device="cuda"); B = torch.randn((N, K) if tb else (K, N), device="cuda")
    C = torch.randn(M, N, device="cuda")
    f = lambda: L.msat_gemm(A.data_ptr(), K, B.data_ptr(), B.shape[1], tb, C.data_ptr(), N, 0, M, N, K, 1, s)
    us = timeit(f)
    print(json.dumps({"what": "gemm " + what, "M": M, "N": N, "K": K, "us": round(us, 1),
                      "tflops": round(2 * M * N * K / us / 1e6, 1)}))
    if tb:  # bf16x3 split GEMM on the same shape (weights pre-split)
        planes = torch.empty(3 * N * K, dtype=torch.int16, device="cuda")
        L.msat_split_bf16x3(B.data_ptr(), N, K, K, planes.data_ptr(), s)
        f3 = lambda: L.msat_gemm_x3(A.data_ptr(), K, planes.data_ptr(), C.data_ptr(), N, 0, M, N, K, 1, s)
        for ti in ("2", "4"):
            os.environ["MARLSAT_GEMM_X3_TI"] = ti
            us = timeit(f3)
            print(json.dumps({"what": f"gemm_x3 ti{ti} " + what, "M": M, "N": N, "K": K, "us": round(us, 1),
                              "tflops": round(2 * M * N * K / us / 1e6, 1)}))
        os.environ.pop("MARLSAT_GEMM_X3_TI")
    del A, B, C
for M, K, N, what in WGRADS:
    A = torch.randn(M, K, device="cuda"); G = torch.randn(M, N, device="cuda"); W = torch.empty(K, N, device="cuda")
    ws = torch.empty(int(L.msat_gemm_wgrad_workspace_bytes(M, K, N)) // 4 + 1, device="cuda")
    f = lambda: L.msat_gemm_wgrad(A.data_ptr(), K, G.data_ptr(), N, W.data_ptr(), N, M, K, N, 1, ws.data_ptr(), s)
    us = timeit(f)
    print(json.dumps({"what": "wgrad " + what, "M": M, "K": K, "N": N, "us": round(us, 1),
                      "tflops": round(2 * M * N * K / us / 1e6, 1)}))
    del A, G, W, ws
