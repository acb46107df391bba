"""Register-A GRU forward microbenchmark: bf16x3 (msat_gru_ln_fused_fwd_x3r) vs fp16x2
(msat_gru_ln_fused_fwd_h2r, incl. its fixup launch) on the encoder's shapes, with and without the
training tape.  Prints one JSON line per (cell, tape, kernel): ms per call, fp32-equivalent TF/s.
    python profiles/gru_r_bench.py [rows_clause rows_var]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import torch  # noqa: E402

from marlsat import _lib  # noqa: E402

H = 128
RC = int(sys.argv[1]) if len(sys.argv) > 1 else 1400000
RV = int(sys.argv[2]) if len(sys.argv) > 2 else 560000
s = _lib.stream_ptr()
L_ = _lib.lib
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
    flop = 2.0 * R * 3 * H * (H + Kx)
    for tape in (False, True):
        gp = g4.data_ptr() if tape else 0
        runs = {
            "x3r": lambda: L_.msat_gru_ln_fused_fwd_x3r(*args, h.data_ptr(), H, pi.data_ptr(), kxp, bi.data_ptr(),
                                                        ph.data_ptr(), bh.data_ptr(), sc.data_ptr(), lb.data_ptr(),
                                                        out.data_ptr(), H, gp, 4 * H, R, H, s),
            "h2r": lambda: L_.msat_gru_ln_fused_fwd_h2r(*args, h.data_ptr(), H, qi.data_ptr(), qh.data_ptr(),
                                                        pi.data_ptr(), ph.data_ptr(), kxp, bi.data_ptr(),
                                                        bh.data_ptr(), sc.data_ptr(), lb.data_ptr(), out.data_ptr(),
                                                        H, gp, 4 * H, R, H, flags.data_ptr(), bad.data_ptr(), s),
        }
        for name, fn in runs.items():
            if name not in os.environ.get("GRU_KERNELS", "x3r,h2r").split(",") or str(tape) not in os.environ.get(
                    "GRU_TAPE", "False,True"):
                continue
            for _ in range(3):
                assert fn() == 0
            torch.cuda.synchronize()
            n = int(os.environ.get("GRU_REPS", "10"))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(n):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / n
            rec = {"cell": cell, "rows": R, "tape": tape, "kernel": name, "ms": round(ms, 4),
                   "tflops_fp32_equiv": round(flop / ms / 1e9, 1),
                   "flagged_tiles": int(flags.sum()) if name == "h2r" else None}
            if os.environ.get("GRU_CHECKSUM"):  # bit checksums of the outputs (A/B builds must agree)
                rec["out_bits"] = int(out.view(torch.int32).to(torch.int64).sum())
                if tape:
                    rec["g4_bits"] = int(g4.view(torch.int32).to(torch.int64).sum())
            print(json.dumps(rec), flush=True)
