"""A GRU cell's dual data gradient (msat_gemm_h2_dual) and dual weight gradient (msat_gemm_wgrad_h2_dual) on
the clause training shape (packed rows D = [dan | dar | daz | dan r], ld 4H): HIP-event time, algorithmic
bytes and GB/s -- for the fp32 packed rows and for the same rows as fp16x2 planes (the *_planes entry points,
round 5), alternated `alt` times on one box.
usage: dual_bench.py [rows] [reps] [input width K1: 256 clause cell, 128 variable cell] [alt]"""
import ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import torch
from marlsat import _lib

L = _lib.lib
M = int(sys.argv[1]) if len(sys.argv) > 1 else 1316000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
H = 128
K1 = int(sys.argv[3]) if len(sys.argv) > 3 else 2 * H
alt = int(sys.argv[4]) if len(sys.argv) > 4 else 1
torch.manual_seed(0)
s = _lib.stream_ptr()
D = torch.randn(M, 4 * H, device="cuda") * 1e-3
m = D.abs().amax(dim=1)
rexp = torch.where(m == 0, torch.full_like(m, 0x3FFF, dtype=torch.int32), 15 - torch.frexp(m)[1]).to(torch.int32)
# the planes buffer: row r = [hi (4H fp16) | lo (4H fp16)] of D[r] 2^rexp[r] (what the GRU backward writes)
pow2 = lambda e: ((e + 127) << 23).view(torch.float32)  # exact 2^e, |e| <= 126
x = D * pow2(rexp.clamp(-120, 120).unsqueeze(1))
hi = x.half()
P = torch.cat([hi, (x - hi.float()).half()], dim=1).contiguous()
del x, hi
planes = []
for n, k, rot in ((H, 3 * H, 0), (K1, 3 * H, 2 * H)):
    W = torch.randn(n, k, device="cuda") * 0.05
    p2 = torch.empty(2 * n * k + 8, dtype=torch.int16, device="cuda")
    p3 = torch.empty(3 * n * k + 8, dtype=torch.int16, device="cuda")
    bad = torch.empty(1, dtype=torch.int32, device="cuda")
    L.msat_split_f16x2_rot(W.data_ptr(), n, k, k, rot, p2.data_ptr(), bad.data_ptr(), s)
    L.msat_split_bf16x3_rot(W.data_ptr(), n, k, k, rot, p3.data_ptr(), s)
    planes.append((W, p2, p3, bad))
dh = torch.randn(M, H, device="cuda")
dx = torch.empty(M, K1, device="cuda")
hx = torch.randn(M, H, device="cuda")
gin = torch.randn(M, K1, device="cuda")
gW0 = torch.zeros(H, 3 * H, device="cuda")
gW1 = torch.zeros(K1, 3 * H, device="cuda")
ws = torch.empty(int(L.msat_gemm_wgrad_dual_workspace_bytes(M, H, 3 * H, K1, 3 * H)) // 4 + 1, device="cuda")
dgh, dgi = D.data_ptr() + 4 * H, D.data_ptr()
pgh, pgi = P.data_ptr() + 2 * H, P.data_ptr()
W0 = (planes[0][1].data_ptr(), planes[0][2].data_ptr(), planes[0][3].data_ptr())
W1 = (planes[1][1].data_ptr(), planes[1][2].data_ptr(), planes[1][3].data_ptr())
fd = lambda: L.msat_gemm_h2_dual(dgh, 4 * H, *W0, dh.data_ptr(), H, H, 1, dgi, 4 * H, *W1, dx.data_ptr(), K1, K1, 0,
                                  rexp.data_ptr(), M, 3 * H, s)
fdp = lambda: L.msat_gemm_h2_dual_planes(pgh, 8 * H, *W0, dh.data_ptr(), H, H, 1, pgi, 8 * H, *W1, dx.data_ptr(), K1,
                                         K1, 0, 4 * H, rexp.data_ptr(), M, 3 * H, s)
fw = lambda: L.msat_gemm_wgrad_h2_dual(hx.data_ptr(), H, dgh, 4 * H, gW0.data_ptr(), 3 * H, H, 3 * H, 0,
                                       gin.data_ptr(), K1, dgi, 4 * H, gW1.data_ptr(), 3 * H, K1, 3 * H, 2 * H,
                                       rexp.data_ptr(), M, 1, ws.data_ptr(), s)
fwp = lambda: L.msat_gemm_wgrad_h2_dual_planes(hx.data_ptr(), H, pgh, 8 * H, gW0.data_ptr(), 3 * H, H, 3 * H, 0,
                                               gin.data_ptr(), K1, pgi, 8 * H, gW1.data_ptr(), 3 * H, K1, 3 * H, 2 * H,
                                               4 * H, rexp.data_ptr(), M, 1, ws.data_ptr(), s)
for a_ in range(alt):
    for name, f, nb in (("dual dgrad", fd, 4.0 * M * (4 * H + 2 * H + K1 + 1)),
                        ("dual dgrad planes", fdp, 4.0 * M * (4 * H + 2 * H + K1 + 1)),
                        ("dual wgrad", fw, 4.0 * M * (H + K1 + 4 * H + 1)),
                        ("dual wgrad planes", fwp, 4.0 * M * (H + K1 + 4 * H + 1))):
        if os.environ.get("DUAL_ONLY") and os.environ["DUAL_ONLY"] not in name:
            continue
        for _ in range(2):
            assert f() == 0
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            f()
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) / reps * 1e3
        rec = {"what": name, "rows": M, "K1": K1, "us": round(us, 1), "algorithmic_bytes": nb,
               "GBps": round(nb / us / 1e3, 1)}
        if os.environ.get("DUAL_CHECKSUM"):  # bit checksums of the outputs (A/B builds must agree)
            outs = (dh, dx) if "dgrad" in name else (gW0, gW1)
            rec["bits"] = [int(o.view(torch.int32).to(torch.int64).sum()) for o in outs]
        print(json.dumps(rec), flush=True)
