"""Diagnostic: where a GRU-forward k step spends its cycles.  Needs a library built from gru_fused.hip with
the s_memtime stamps of profiles/archive_r03/gru_stamp.patch (MARLSAT_LIB=...), which adds
msat_debug_gru_stamps.  Runs the fp16x2 kernel on the encoder's clause / var shapes (tape on and off) and
prints each phase's share of the wave's cycles, averaged over the launch's waves (shares only: the stamps'
waits forbid overlaps the real kernel has).  usage: gru_stamps.py [rows_clause rows_var]"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import torch  # noqa: E402

from marlsat import _lib  # noqa: E402

H = 128
RC = int(sys.argv[1]) if len(sys.argv) > 1 else 1400000
RV = int(sys.argv[2]) if len(sys.argv) > 2 else 560000
L_ = _lib.lib
L_.msat_debug_gru_stamps.restype = ctypes.c_int
L_.msat_debug_gru_stamps.argtypes = [ctypes.c_void_p]
s = _lib.stream_ptr()
SEG, CAP = 8, 16384 * 8
names = ["prologue", "early DMA issue", "MFMA blocks", "vmcnt wait", "barrier", "output flush", "loop+epilogue", "steps"]
for cell, R, segs_w, segs_ld in (("clause", RC, (2 * H, 4), (2 * H, 4)), ("var", RV, (H, 8), (2 * H, 8))):
    g = torch.Generator(device="cuda").manual_seed(0)
    X = [torch.randn(R, ld, device="cuda", generator=g) for ld in segs_ld]
    h = torch.randn(R, H, device="cuda", generator=g)
    Kx = sum(segs_w)
    kxp = (Kx + 31) // 32 * 32
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
    pi = torch.empty(3 * 3 * H * kxp + 8, dtype=torch.int16, device="cuda")
    ph = torch.empty(3 * 3 * H * H + 8, dtype=torch.int16, device="cuda")
    qi = torch.empty(2 * 3 * H * kxp + 8, dtype=torch.int16, device="cuda")
    qh = torch.empty(2 * 3 * H * H + 8, dtype=torch.int16, device="cuda")
    bad = torch.zeros(2, dtype=torch.int32, device="cuda")
    flags = torch.zeros((R + 127) // 128, dtype=torch.int32, device="cuda")
    L_.msat_split_bf16x3_t(wi.data_ptr(), Kx, 3 * H, 3 * H, kxp, pi.data_ptr(), s)
    L_.msat_split_bf16x3_t(wh.data_ptr(), H, 3 * H, 3 * H, H, ph.data_ptr(), s)
    L_.msat_split_f16x2_t(wi.data_ptr(), Kx, 3 * H, 3 * H, kxp, qi.data_ptr(), bad.data_ptr(), s)
    L_.msat_split_f16x2_t(wh.data_ptr(), H, 3 * H, 3 * H, H, qh.data_ptr(), bad.data_ptr() + 4, s)
    for tape in (False, True):
        gp = g4.data_ptr() if tape else 0
        for _ in range(3):  # the last launch's stamps are read
            assert L_.msat_gru_ln_fused_fwd_h2r(*args, h.data_ptr(), H, qi.data_ptr(), qh.data_ptr(), pi.data_ptr(),
                                                ph.data_ptr(), kxp, bi.data_ptr(), bh.data_ptr(), sc.data_ptr(),
                                                lb.data_ptr(), out.data_ptr(), H, gp, 4 * H, R, H, flags.data_ptr(),
                                                bad.data_ptr(), s) == 0
        torch.cuda.synchronize()
        buf = np.zeros(CAP * SEG, dtype=np.uint64)
        assert L_.msat_debug_gru_stamps(buf.ctypes.data) == 0
        st = buf.reshape(CAP, SEG)[: min(CAP, ((R + 127) // 128) * 8)].astype(np.float64)
        total = st[:, 0] + st[:, 6]
        epi = st[:, 6] - st[:, 1:5].sum(1) - st[:, 5]
        share = {n: float((st[:, k] / total).mean()) for k, n in enumerate(names[:6])}
        share["epilogue (gates, LN, tape, stage)"] = float((epi / total).mean())
        print(json.dumps({"cell": cell, "rows": R, "tape": tape, "steps_per_tile": float(st[:, 7].mean()),
                          "wave_cycles_per_tile": float(total.mean()),
                          "cycles_per_step": float((st[:, 1:5].sum(1) / st[:, 7]).mean()),
                          "shares": {k: round(v, 4) for k, v in share.items()}}), flush=True)
