"""Fused GRU + LayerNorm forward microbenchmark (rollout = no tape, training = with the G4 tape):
row split RS=1 (2 waves/SIMD, 128 accumulators per lane) vs RS=2 (4 waves/SIMD, 64)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import torch
from marlsat import _lib

H = 128
# bench training shapes (uf50, micro-batch 1,366): var cells read [gathered half (ld 2H) | vfeat (8)],
# the clause cell [gathered (2H) | counts (4)]
for kind, R, segs_w, segs_ld in (("var", 407000, (H, 8), (2 * H, 8)), ("clause", 1036000, (2 * H, 4), (2 * H, 4))):
    g = torch.Generator(device="cuda").manual_seed(0)
    X = [torch.randn(R, ld, device="cuda", generator=g) for ld in segs_ld]
    h = torch.randn(R, H, device="cuda", generator=g)
    Kx = sum(segs_w)
    wi = torch.randn(Kx, 3 * H, device="cuda", generator=g) / Kx ** 0.5
    wh = torch.randn(H, 3 * H, device="cuda", generator=g) / H ** 0.5
    bi, bh = torch.zeros(3 * H, device="cuda"), torch.zeros(3 * H, device="cuda")
    sc, lb = torch.ones(H, device="cuda"), torch.zeros(H, device="cuda")
    out = torch.empty(R, H, device="cuda")
    g4 = torch.empty(R, 4 * H, device="cuda")
    args = []
    for x, w in zip(X, segs_w):
        args += [x.data_ptr(), x.shape[1], w]
    args += [0, 0, 0] * (3 - len(segs_w))
    Kp = (Kx + 15) // 16 * 16
    wiT = torch.empty(3 * H, Kp, device="cuda"); whT = torch.empty(3 * H, H, device="cuda")
    _lib.lib.msat_transpose_pad(wi.data_ptr(), Kx, 3 * H, 3 * H, wiT.data_ptr(), Kp, _lib.stream_ptr())
    _lib.lib.msat_transpose_pad(wh.data_ptr(), H, 3 * H, 3 * H, whT.data_ptr(), H, _lib.stream_ptr())
    kxp = Kp
    wip = torch.zeros(kxp, 3 * H, device="cuda"); wip[:Kx] = wi
    pi = torch.empty(3 * kxp * 3 * H + 8, dtype=torch.int16, device="cuda")
    ph = torch.empty(3 * H * 3 * H + 8, dtype=torch.int16, device="cuda")
    _lib.lib.msat_split_bf16x3(wip.data_ptr(), kxp, 3 * H, 3 * H, pi.data_ptr(), _lib.stream_ptr())
    _lib.lib.msat_split_bf16x3(wh.data_ptr(), H, 3 * H, 3 * H, ph.data_ptr(), _lib.stream_ptr())
    for tape in (False, True):
        for rs in ("2", "x3"):
            os.environ["MARLSAT_GRU_RS"] = rs if rs in ("1", "2") else "2"
            if rs.startswith("x3"):
                f = lambda: _lib.lib.msat_gru_ln_fused_fwd_x3(*args, h.data_ptr(), H, pi.data_ptr(), kxp, bi.data_ptr(),
                                                              ph.data_ptr(), bh.data_ptr(), sc.data_ptr(),
                                                              lb.data_ptr(), out.data_ptr(), H,
                                                              g4.data_ptr() if tape else 0, 4 * H, R, H,
                                                              _lib.stream_ptr())
            elif rs == "t":
                f = lambda: _lib.lib.msat_gru_ln_fused_fwd_t(*args, h.data_ptr(), H, wiT.data_ptr(), bi.data_ptr(),
                                                             whT.data_ptr(), bh.data_ptr(), sc.data_ptr(),
                                                             lb.data_ptr(), out.data_ptr(), H,
                                                             g4.data_ptr() if tape else 0, 4 * H, R, H,
                                                             _lib.stream_ptr())
            else:
                f = lambda: _lib.lib.msat_gru_ln_fused_fwd(*args, h.data_ptr(), H, wi.data_ptr(), bi.data_ptr(),
                                                           wh.data_ptr(), bh.data_ptr(), sc.data_ptr(), lb.data_ptr(),
                                                           out.data_ptr(), H, g4.data_ptr() if tape else 0, 4 * H, R,
                                                           H, _lib.stream_ptr())
            f(); torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                f()
            b.record(); torch.cuda.synchronize()
            us = a.elapsed_time(b) / 10 * 1e3
            fl = 2 * R * 3 * H * (H + (Kx + 15) // 16 * 16)
            print(json.dumps({"cell": kind, "R": R, "tape": tape, "RS": rs, "us": round(us, 1),
                              "tflops": round(fl / us / 1e6, 1)}))
