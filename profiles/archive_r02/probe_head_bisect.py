"""Probe (not collected): which backward stage differs between the fp64- and fp32-folded forward."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "marl-sat_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tests.test_gnn_gpu import _setup  # noqa: E402


def main():
    torch.cuda.set_device(0)
    net, b, P, batch, av, am, A, M = _setup(50, 218, 10, 128, 16, 4, 0, seed=11)
    g = torch.Generator(device="cuda").manual_seed(5)
    res = {}
    for mode in ("0", "1"):
        os.environ["MARLSAT_FOLD_F64"] = mode
        logits, value, state = net.forward(b, save=True)
        Hp, Hn, Hc, tape, ht = state
        dl = torch.where(torch.isfinite(logits), torch.randn(logits.shape, device="cuda", generator=g.manual_seed(1)),
                         torch.zeros_like(logits)).contiguous()
        dv = torch.randn(value.shape, device="cuda", generator=g.manual_seed(2)).contiguous()
        net.grads.zero_()
        dHp, dHn, dHc = torch.zeros_like(Hp), torch.zeros_like(Hn), torch.zeros_like(Hc)
        net.critic_head_backward(b, Hp, Hn, Hc, ht, dv, dHp, dHn, dHc)
        g_crit = net.grads.clone()
        net.actor_head_backward(b, ht, dl, dHp, dHn, dHc)
        g_head = net.grads.clone()
        res[mode] = dict(logits=logits.clone(), Hp=Hp.clone(), Hn=Hn.clone(), Hc=Hc.clone(), g_crit=g_crit,
                         g_head=g_head, dHp=dHp.clone(), dHn=dHn.clone(), dHc=dHc.clone(),
                         **{f"ht_{k}": v.clone() for k, v in vars(ht).items() if torch.is_tensor(v)})
    a, c = res["0"], res["1"]
    for k in a:
        d = (a[k] - c[k]).abs()
        fin = torch.isfinite(d)
        print(f"{k:10s} shape {tuple(a[k].shape)} max|diff| {float(d[fin].max()) if fin.any() else 0:.3e} "
              f"max|val| {float(a[k][torch.isfinite(a[k])].abs().max()):.3e} nonfinite {int((~fin).sum())}")
    tab = net.tab
    d = (a["g_head"] - c["g_head"]).abs().cpu().numpy()
    for name, (o, shp) in sorted(tab.items(), key=lambda t: t[1][0]):
        n = int(np.prod(shp))
        if d[o:o + n].max() > 1e-4:
            print("head-grad diff", name, float(d[o:o + n].max()))


if __name__ == "__main__":
    main()
