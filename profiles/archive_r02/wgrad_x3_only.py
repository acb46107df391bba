"""bf16x3 weight gradient (msat_gemm_wgrad default path) on the uf50 training shapes, HIP-event timed.
usage: wgrad_x3_only.py [reps]   (MARLSAT_WGRAD_WG sets the workgroup budget)"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import torch
from marlsat import _lib

L = _lib.lib
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
Nv, Nc, H = 407000, 1036000, 128
s = _lib.stream_ptr()
for M, K, N, what in [(Nv, H, 3 * H, "var"), (Nc, H, 3 * H, "clause dWh"), (Nc, 2 * H, 3 * H, "clause dF")]:
    A = torch.randn(M, K, device="cuda"); G = torch.randn(M, N, device="cuda"); W = torch.empty(K, N, device="cuda")
    ws = torch.empty(int(L.msat_gemm_wgrad_workspace_bytes(M, K, N)) // 4 + 1, device="cuda")
    f = lambda: L.msat_gemm_wgrad(A.data_ptr(), K, G.data_ptr(), N, W.data_ptr(), N, M, K, N, 0, ws.data_ptr(), s)
    f(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        f()
    b.record(); torch.cuda.synchronize()
    us = a.elapsed_time(b) / reps * 1e3
    print(json.dumps({"what": what, "M": M, "K": K, "N": N, "wg": os.environ.get("MARLSAT_WGRAD_WG", "default"),
                      "us": round(us, 1), "tflops": round(2 * M * N * K / us / 1e6, 1)}))
