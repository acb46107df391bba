"""Probe (not collected): x3r / h2r GRU kernel determinism and error vs the fp64 reference."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "marl-sat_amd"))
import torch
from tests.test_gru_fused_gpu import _fwd, _ref_gru_ln, _setup
torch.cuda.set_device(0)
for kind in ("var", "clause4"):
    for R in (1, 128, 1000):
        segs, x, h, wi, bi, wh, bh, sc, lb = _setup(R, 128, kind, seed=R + 128)
        d = lambda t: t.double()
        ref, _, _ = _ref_gru_ln(d(x), d(h), d(wi), d(bi), d(wh), d(bh), d(sc), d(lb), 128)
        for lay in ("x3r", "h2r"):
            outs = []
            for tape in (True, False, True, False):
                g4 = torch.full((R, 512), float("nan"), device="cuda") if tape else None
                outs.append(_fwd(segs, h, wi, bi, wh, bh, sc, lb, R, 128, g4, lay).clone())
            e = [float((o.double() - ref).abs().max()) for o in outs]
            same = [torch.equal(outs[0], o) for o in outs]
            bad_rows = int(((outs[1].double() - ref).abs().amax(1) > 1e-3).sum())
            print(kind, R, lay, "err", ["%.2e" % v for v in e], "equal-to-first", same, "bad rows (no tape)", bad_rows, flush=True)
