"""GEMM / weight-gradient microbenchmark on the MAPPO network's dominant shapes: register-staged
kernels (MARLSAT_GEMM=1) vs the LDS-DMA fast path, HIP-event timed, TFLOP/s vs fp32 MFMA peak."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import torch
from marlsat import _lib

L = _lib.lib
GEMMS = [  # M, N, K, transB  (what)
    (887000, 128, 128, 0, "fwd phi_c (var rows)"), (857000, 256, 128, 0, "fwd phi_v (clause rows)"),
    (221000, 128, 384, 1, "bwd dh = dGh Wh^T"), (221000, 128, 384, 1, "bwd dX = dGi Wi^T"),
    (214000, 256, 384, 1, "bwd dGIN = dGi Wic^T"), (221000, 128, 128, 1, "bwd phi^T"),
]
WGRADS = [(221000, 128, 384, "dWh / dWi"), (214000, 256, 384, "dWi_c"), (221000, 128, 128, "dphi")]


def timeit(fn, reps=10):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3  # us


res = []
for M, N, K, tb, what in GEMMS:
    A = torch.randn(M, K, device="cuda"); B = torch.randn((N, K) if tb else (K, N), device="cuda")
    C = torch.empty(M, N, device="cuda"); bias = torch.randn(N, device="cuda")
    s = _lib.stream_ptr()
    f = lambda: L.msat_gemm(A.data_ptr(), K, B.data_ptr(), B.shape[1], tb, C.data_ptr(), N, bias.data_ptr(), M, N, K, 0, s)
    row = {"what": what, "M": M, "N": N, "K": K, "transB": tb}
    for tag, env, d in (("old", "1", "32"), ("d32", "0", "32"), ("d16", "0", "16"), ("nostore16", "2", "16")):
        os.environ["MARLSAT_GEMM"] = env
        os.environ["MARLSAT_GEMM_D"] = d
        us = timeit(f)
        row[tag + "_us"] = round(us, 1)
        row[tag + "_tflops"] = round(2 * M * N * K / us / 1e6, 1)
    res.append(row)
os.environ["MARLSAT_GEMM"] = "0"
for M, K, N, what in WGRADS:
    A = torch.randn(M, K, device="cuda"); G = torch.randn(M, N, device="cuda"); W = torch.empty(K, N, device="cuda")
    ws = torch.empty(int(L.msat_gemm_wgrad_workspace_bytes(M, K, N)) // 4 + 1, device="cuda")
    s = _lib.stream_ptr()
    f = lambda: L.msat_gemm_wgrad(A.data_ptr(), K, G.data_ptr(), N, W.data_ptr(), N, M, K, N, 0, ws.data_ptr(), s)
    row = {"what": "wgrad " + what, "M": M, "K": K, "N": N}
    for tag, env, d in (("old", "1", "32"), ("d32", "0", "32"), ("d16", "0", "16")):
        os.environ["MARLSAT_GEMM"] = env
        os.environ["MARLSAT_GEMM_D"] = d
        us = timeit(f)
        row[tag + "_us"] = round(us, 1)
        row[tag + "_tflops"] = round(2 * M * N * K / us / 1e6, 1)
    res.append(row)
for r in res:
    print(json.dumps(r))
