"""GRU + LayerNorm backward from the tape (msat_gru_ln_bwd_g4f, packed rows, dh assigned, gate-bias and
feature partials) on the uf50 training shapes, HIP-event timed, with its HBM rate.
usage: gru_bwd_only.py [reps]   (BWD_ALT=n alternates the fp32-row and planes forms n times)
Measured: var 507 us (4.5 TB/s), clause 1067 us (5.5 TB/s); more blocks, two rows per wave with
all loads first (3 / 2 waves per SIMD instead of 5 / 4), or the next row's loads issued before this
row's stores (4 / 3 waves per SIMD: 567 / 1249 vs 526 / 1141 us) measured slower."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import torch
from marlsat import _lib

L = _lib.lib
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
H = 128
s = _lib.stream_ptr()
for what, R, nf, ldf in [("var", 407000, 6, 8), ("clause", 1036000, 2, 4)]:
    r = lambda *sh: torch.randn(*sh, device="cuda")
    dy, g4, hp, feat = r(R, H), r(R, 4 * H), r(R, H), r(R, ldf)
    sc, dln = r(H), torch.zeros(2 * H, device="cuda")
    dG, dh = torch.empty(R, 4 * H, device="cuda"), torch.empty(R, H, device="cuda")
    dbi, dbh, dfeat = torch.zeros(3 * H, device="cuda"), torch.zeros(H, device="cuda"), torch.zeros(nf * 3 * H, device="cuda")
    part = torch.empty(int(L.msat_gru_ln_bwd_partial_floats(R, H)), device="cuda")
    rexp = torch.empty(R, dtype=torch.int32, device="cuda")
    # forms: "e" the packed fp32 rows + row exponents (flags 7), "p" the same rows as fp16x2 planes (flags 15)
    for alt in range(int(os.environ.get("BWD_ALT", "1"))):
        for form, flags in (("e", 0b111), ("p", 0b1111)):
            f = lambda: L.msat_gru_ln_bwd_g4fe(dy.data_ptr(), H, g4.data_ptr(), 4 * H, hp.data_ptr(), H, sc.data_ptr(),
                                               dG.data_ptr(), 4 * H, dG.data_ptr() + 4 * H, 4 * H, dh.data_ptr(), H,
                                               dln.data_ptr(), dln.data_ptr() + 4 * H, dbi.data_ptr(), dbh.data_ptr(),
                                               feat.data_ptr(), ldf, nf, dfeat.data_ptr(), part.data_ptr(), R, H, flags,
                                               rexp.data_ptr(), s)
            assert f() == 0
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(reps):
                f()
            b.record(); torch.cuda.synchronize()
            us = a.elapsed_time(b) / reps * 1e3
            nbytes = R * 4 * (H + 4 * H + H + nf + 4 * H + H + 1)  # dy, tape, h, feat in; packed dG, dh, rexp out
            print(json.dumps({"what": what, "form": form, "R": R, "us": round(us, 1),
                              "GBps": round(nbytes / us / 1e3, 1)}), flush=True)
