"""Accuracy of the GRU forward kernels' gate pre-activations (the tape [r | z | gin | ghn]) against float64, per
element relative to the sum of its terms' magnitudes (|x| |Wi| + |h| |Wh| + |b|): the fp32 MFMA kernel ("plain"),
the bf16x3 register-A kernel (x3r) and the fp16x2 kernel (h2r, the default), on the encoder's var and clause
shapes with realistic magnitudes (LayerNorm-like h, gathered sums as inputs, small static features).  Run it once
per library build (MARLSAT_LIB) to compare fp16x2 variants (profiles/gpu_r06/r06d.sh).

    python profiles/gru_h2_accuracy.py [R]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "marl-sat_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

from test_gru_fused_gpu import _fwd, _ref_gru_ln, _setup  # noqa: E402


def realistic(kind, R, H, seed):
    segs, x, h, wi, bi, wh, bh, sc, lb = _setup(R, H, kind, seed)
    g = torch.Generator(device="cuda").manual_seed(seed + 1)
    if kind == "var8":  # [gathered sum of ~6 clause states | x, deg+/C, deg-/C, 0, n+, n-, 0, 0]
        NV, _, _, _ = segs[0]
        NV.mul_(2.5)
        vf = segs[1][0]
        vf.zero_()
        vf[:, 0] = torch.randint(0, 2, (R,), device="cuda", generator=g).float()
        vf[:, 1] = torch.rand(R, device="cuda", generator=g) * 0.06
        vf[:, 2] = torch.rand(R, device="cuda", generator=g) * 0.06
        vf[:, 4] = torch.randint(0, 14, (R,), device="cuda", generator=g).float()
        vf[:, 5] = torch.randint(0, 14, (R,), device="cuda", generator=g).float()
        x = torch.cat([NV[:, :H], vf], 1)
    else:  # clause4: [sum of <= 3 var states (2H) | n+, n-, 0, 0]
        GIN = segs[0][0]
        GIN.mul_(1.7)
        cd = segs[1][0]
        cd.zero_()
        cd[:, 0] = torch.randint(0, 4, (R,), device="cuda", generator=g).float()
        cd[:, 1] = 3 - cd[:, 0]
        x = torch.cat([GIN, cd], 1)
    return segs, x, h, wi, bi, wh, bh, sc, lb


def stats(kind, R, H=128):
    segs, x, h, wi, bi, wh, bh, sc, lb = realistic(kind, R, H, seed=17)
    d = lambda t: t.double()
    ref, gi, gh = _ref_gru_ln(d(x), d(h), d(wi), d(bi), d(wh), d(bh), d(sc), d(lb), H)
    tape_ref = torch.cat([gi[:, :H] + gh[:, :H], gi[:, H:2 * H] + gh[:, H:2 * H], gi[:, 2 * H:], gh[:, 2 * H:]], 1)
    absx = torch.cat([d(x).abs() @ d(wi).abs() + d(bi).abs(), d(h).abs() @ d(wh).abs() + d(bh).abs()], 1)
    ab = torch.cat([absx[:, :H] + absx[:, 3 * H:4 * H], absx[:, H:2 * H] + absx[:, 4 * H:5 * H],
                    absx[:, 2 * H:3 * H], absx[:, 5 * H:]], 1)
    out = {}
    for lay in ("plain", "x3r", "h2r"):
        g4 = torch.empty(R, 4 * H, device="cuda")
        o = _fwd(segs, h, wi, bi, wh, bh, sc, lb, R, H, g4, lay)
        rel = ((g4.double() - tape_ref).abs() / ab).flatten()
        q = torch.quantile(rel[torch.randperm(rel.numel(), device="cuda")[:1 << 20]],
                           torch.tensor([0.5, 0.99], dtype=torch.float64, device="cuda")).tolist()
        oe = (o.double() - ref).abs()
        out[lay] = (q[0], q[1], float(rel.max()), float(rel.mean()), float(oe.mean()), float(oe.max()))
    return out


if __name__ == "__main__":
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 70000
    print(f"lib {os.environ.get('MARLSAT_LIB', 'libmarlsat.so')}: tape error / sum|terms| (median, p99, max, mean); "
          f"h' error (mean, max)")
    for kind in ("var8", "clause4"):
        for lay, (m, p99, mx, mean, om, ox) in stats(kind, R).items():
            print(f"  {kind:8s} {lay:5s}: tape median {m:.3g} p99 {p99:.3g} max {mx:.3g} mean {mean:.3g} | "
                  f"h' mean {om:.3g} max {ox:.3g}", flush=True)
