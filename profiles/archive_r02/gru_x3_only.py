"""x3 fused GRU forward on the uf50 training shapes only (for PMC passes / A/B timing).
usage: python profiles/gru_x3_only.py [reps] [cells]   cells: var,clause"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import torch
from marlsat import _lib

H = 128
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
cells = (sys.argv[2] if len(sys.argv) > 2 else "var,clause").split(",")
shapes = {"var": (407000, (H, 8), (2 * H, 8)), "clause": (1036000, (2 * H, 4), (2 * H, 4))}
for kind in cells:
    R, segs_w, segs_ld = shapes[kind]
    g = torch.Generator(device="cuda").manual_seed(0)
    X = [torch.randn(R, ld, device="cuda", generator=g) for ld in segs_ld]
    h = torch.randn(R, H, device="cuda", generator=g)
    Kx = sum(segs_w)
    kxp = (Kx + 15) // 16 * 16
    wip = torch.zeros(kxp, 3 * H, device="cuda")
    wip[:Kx] = torch.randn(Kx, 3 * H, device="cuda", generator=g) / Kx ** 0.5
    wh = torch.randn(H, 3 * H, device="cuda", generator=g) / H ** 0.5
    bi, bh = torch.zeros(3 * H, device="cuda"), torch.zeros(3 * H, device="cuda")
    sc, lb = torch.ones(H, device="cuda"), torch.zeros(H, device="cuda")
    out = torch.empty(R, H, device="cuda")
    g4 = torch.empty(R, 4 * H, device="cuda")
    args = []
    for x, w in zip(X, segs_w):
        args += [x.data_ptr(), x.shape[1], w]
    args += [0, 0, 0] * (3 - len(segs_w))
    pi = torch.empty(3 * kxp * 3 * H + 8, dtype=torch.int16, device="cuda")
    ph = torch.empty(3 * H * 3 * H + 8, dtype=torch.int16, device="cuda")
    fn = _lib.lib.msat_gru_ln_fused_fwd_x3
    if os.environ.get("MARLSAT_GRU_LAYOUT") == "x3r":  # register-A kernel: W^T planes, K padded to 32
        kxp = (Kx + 31) // 32 * 32
        pi = torch.empty(3 * kxp * 3 * H + 8, dtype=torch.int16, device="cuda")
        _lib.lib.msat_split_bf16x3_t(wip.data_ptr(), Kx, 3 * H, 3 * H, kxp, pi.data_ptr(), _lib.stream_ptr())
        _lib.lib.msat_split_bf16x3_t(wh.data_ptr(), H, 3 * H, 3 * H, H, ph.data_ptr(), _lib.stream_ptr())
        fn = _lib.lib.msat_gru_ln_fused_fwd_x3r
    else:
        _lib.lib.msat_split_bf16x3(wip.data_ptr(), kxp, 3 * H, 3 * H, pi.data_ptr(), _lib.stream_ptr())
        _lib.lib.msat_split_bf16x3(wh.data_ptr(), H, 3 * H, 3 * H, ph.data_ptr(), _lib.stream_ptr())
    for tape in (False, True):
        f = lambda: fn(*args, h.data_ptr(), H, pi.data_ptr(), kxp, bi.data_ptr(),
                                                      ph.data_ptr(), bh.data_ptr(), sc.data_ptr(), lb.data_ptr(),
                                                      out.data_ptr(), H, g4.data_ptr() if tape else 0, 4 * H, R, H,
                                                      _lib.stream_ptr())
        f(); torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            f()
        b.record(); torch.cuda.synchronize()
        us = a.elapsed_time(b) / reps * 1e3
        fl = 2 * R * 3 * H * (H + kxp)
        print(json.dumps({"cell": kind, "R": R, "tape": tape, "us": round(us, 1), "tflops": round(fl / us / 1e6, 1)}))
