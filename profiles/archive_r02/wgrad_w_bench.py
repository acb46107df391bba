"""Weight-gradient kernels on the training shapes, HIP-event timed: the 128 x 128 tile bf16x3 kernel
(MARLSAT_WGRAD_W=0) against the whole-row kernel (wgrad_x3w_kernel, default), both + the fixed-order
reduce.  G is read from the packed backward rows (ld 4H) as in gnn.py; the dF call rotates by 2H.
Also checks the two agree to the fp32 bound against fp64.
usage: wgrad_w_bench.py [reps]"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import torch
from marlsat import _lib

L = _lib.lib
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
Nv, Nc, H = 407000, 1036000, 128
s = _lib.stream_ptr()
for M, K, what, rot in [(Nv, H, "var dWh", 0), (Nv, H, "var dF (rot)", 2 * H), (Nc, H, "clause dWh", 0),
                        (Nc, 2 * H, "clause dF (rot)", 2 * H)]:
    N = 3 * H
    A = torch.randn(M, K, device="cuda")
    D = torch.randn(M, 4 * H, device="cuda")
    G = D[:, H:] if rot == 0 else D[:, :3 * H]
    W = torch.empty(K, N, device="cuda")
    ws = torch.empty(int(L.msat_gemm_wgrad_workspace_bytes(M, K, N)) // 4 + 1, device="cuda")
    f0 = lambda: L.msat_gemm_wgrad_rot(A.data_ptr(), K, G.data_ptr(), 4 * H, W.data_ptr(), N, M, K, N, rot, 0,
                                      ws.data_ptr(), s)
    res = {}
    m = D.abs().amax(dim=1)
    rexp = torch.where(m == 0, torch.full_like(m, 0x3FFF, dtype=torch.int32), 15 - torch.frexp(m)[1]).to(torch.int32)
    fh = lambda: L.msat_gemm_wgrad_h2(A.data_ptr(), K, G.data_ptr(), 4 * H, rexp.data_ptr(), W.data_ptr(), N, M, K, N,
                                      rot, 0, ws.data_ptr(), s)
    for path in os.environ.get("WGRAD_PATHS", "0,1,1i,h2").split(","):
        os.environ["MARLSAT_WGRAD_W"] = "0" if path == "0" else "1"
        os.environ["MARLSAT_WGRAD_WI"] = "0" if path == "1" else "1"
        f = fh if path == "h2" else f0
        f(); torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            f()
        b.record(); torch.cuda.synchronize()
        us = a.elapsed_time(b) / reps * 1e3
        res[path] = (us, W.clone())
        hbm = M * (K + N) * 4 / (us * 1e-6) / 1e9
        print(json.dumps({"what": what, "M": M, "K": K, "N": N, "kernel": {"0": "x3", "1": "x3w", "1i": "x3w interleaved", "h2": "h2w (fp16x2)"}[path],
                          "us": round(us, 1), "tflops_fp32_equiv": round(2 * M * N * K / us / 1e6, 1),
                          "operand_GBps": round(hbm, 1)}), flush=True)
    ref = torch.roll(A.double().t() @ G.double(), rot, dims=1)
    absprod = torch.roll(A.double().abs().t() @ G.double().abs(), rot, dims=1)
    for path, (_, Wk) in res.items():
        r = float(((Wk.double() - ref).abs() / absprod).max())
        print(json.dumps({"what": what, "kernel": path, "max_err_over_sum_abs": r}))
    del A, D, W, ws
    torch.cuda.empty_cache()
