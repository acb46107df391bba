"""How large is fp32's own noise at the train-cycle test's worst gradient elements?  (verdict r05 item 1)

The teacher-forced train-cycle test (tests/test_mappo_gpu.py) bars every gradient element at
1e-5 |ref| + 4 E32 (+ kink), with E32 the larger error, over the tensor, of two fp32 runs of the oracle that
differ only in the minibatch's row order -- so both share every per-sample sum order.  This script reloads the
inputs the test saw (MARLSAT_PARITY_DUMP=<dir>, written on the GPU box) and runs the fp32 oracle under further
orders of the same sums: variables and clauses relabelled inside every sample (agent variable lists mapped
along, so the function is the same), which changes the order of every sum over variables or clauses (message
passing, pools).  Per step it prints, for the tensors nearest their bar: the device's error at the worst
element, the test's E32, and the fp32 errors at that element and over the tensor under each relabelling.

    python profiles/parity_orderings.py <dump.npz> [n_orders] [steps]     (CPU; oracle only)
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "marl-sat_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

from oracle import net as onet  # noqa: E402

from marlsat.learners import params as Pm  # noqa: E402


def cfg_of(shape):
    V, C, vpa, H, L, mode, T, B, MB, E = (int(v) for v in shape)
    # tests/test_mappo_gpu.py _cfg with the case's overrides
    return dict(NUM_ENVS=B, NUM_STEPS=T, NUM_UPDATES=10, UPDATE_EPOCHS=E, MINIBATCH_SIZE=MB, LEARNING_RATE=3e-3,
                GAMMA=0.995, GAE_LAMBDA=0.95, CLIP_EPS=0.12, ENT_COEF=0.005, VF_COEF=0.5, VF_CLIP=0.5, ANNEAL_LR=True,
                LR_START_FACTOR=1.0, LR_END_FLOOR=2e-5, GNN_HIDDEN_DIM=H, GNN_NUM_MESSAGE_PASSING_STEPS=L,
                action_mode=mode)


def grads(P_np, mb, cfg, av, am, mode, L, dt, log=False):
    Pk = {k: torch.tensor(v, dtype=dt, requires_grad=True) for k, v in P_np.items()}
    mbk = {k: (v.to(dt) if v.is_floating_point() else v) for k, v in mb.items()}
    onet.RELU_LOG = lg = [] if log else None
    try:
        total, _, _, _ = onet.ppo_loss(Pk, L, mbk, cfg, av, am, mode)
    finally:
        onet.RELU_LOG = None
    kink = onet.kink_bound(total, Pk, lg)[0] if log else None
    total.backward()
    return {k: (p.grad.double().numpy() if p.grad is not None else np.zeros(p.shape)) for k, p in Pk.items()}, kink


def relabel(mb, av, rng):
    """The same minibatch with variables and clauses relabelled in every sample (one permutation each, shared by
    the samples so the agent lists stay one table)."""
    V, C = mb["A_pos"].shape[-2:]
    pv, pc = torch.from_numpy(rng.permutation(V)), torch.from_numpy(rng.permutation(C))
    inv = torch.empty_like(pv)
    inv[pv] = torch.arange(V)  # new index of old variable v
    out = dict(mb)
    out["svf"], out["x"] = mb["svf"][:, pv], mb["x"][:, pv]
    out["cf"] = mb["cf"][:, pc]
    out["A_pos"], out["A_neg"] = mb["A_pos"][:, pv][:, :, pc], mb["A_neg"][:, pv][:, :, pc]
    av2 = torch.where(av >= 0, inv[av.clamp(min=0)], av)
    return out, av2


def main():
    path = sys.argv[1]
    n_orders = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    d = np.load(path)
    shape = d["shape"]
    V, C, vpa, H, L, mode, T, B, MB, E = (int(v) for v in shape)
    A = int(d["av"].shape[0])
    M = int(d["av"].shape[1])
    steps = [int(s) for s in sys.argv[3].split(",")] if len(sys.argv) > 3 else \
        sorted(int(k[6:]) for k in d.files if k.startswith("params_"))
    cfg = cfg_of(shape)
    av, am = torch.from_numpy(d["av"].astype(np.int64)), torch.from_numpy(d["am"])
    full = {k[5:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("full_")}
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    print(f"{os.path.basename(path)}: V{V} C{C} A{A} H{H} L{L}, {n_orders} relabellings", flush=True)
    for s in steps:
        idx = d[f"idx_{s}"]
        mb = {k: v[idx] for k, v in full.items()}
        P = Pm.to_flax(d[f"params_{s}"].astype(np.float32), H, L, A, M, mode, 16)
        gdev = Pm.to_flax(d[f"grads_{s}"].astype(np.float32), H, L, A, M, mode, 16)
        g64, kink = grads(P, mb, cfg, av, am, mode, L, torch.float64, log=True)
        g32, _ = grads(P, mb, cfg, av, am, mode, L, torch.float32)
        rows = torch.from_numpy(np.arange(len(idx))[::-1].copy())
        g32r, _ = grads(P, {k: v[rows] for k, v in mb.items()}, cfg, av, am, mode, L, torch.float32)
        rng = np.random.default_rng(1000 + s)
        gperm = []
        for i in range(n_orders):
            mbp, avp = relabel(mb, av, rng)
            gperm.append(grads(P, mbp, cfg, avp, am, mode, L, torch.float32)[0])
            print(f"  step {s}: relabelling {i + 1}/{n_orders} done", flush=True)
        ratios = {}
        for k in g64:
            ref = g64[k]
            e32 = max(np.abs(g32[k] - ref).max(), np.abs(g32r[k] - ref).max())
            kb = np.broadcast_to(np.asarray(kink[k], np.float64), ref.shape)
            err = np.abs(np.asarray(gdev[k], np.float64) - ref)
            r = err / np.maximum(1e-5 * np.abs(ref) + 4 * e32 + kb, 1e-300)
            ratios[k] = (float(r.max()), int(np.argmax(r)), e32)
        for k, (rmax, iw, e32) in sorted(ratios.items(), key=lambda kv: -kv[1][0])[:5]:
            ref = g64[k]
            dev_e = abs(float(np.asarray(gdev[k]).flat[iw]) - float(ref.flat[iw]))
            el = [abs(g[k].flat[iw] - ref.flat[iw]) for g in gperm]
            tens = [np.abs(g[k] - ref).max() for g in gperm]
            e32_all = max([e32] + tens)
            r_all = float((np.abs(np.asarray(gdev[k], np.float64) - ref) /
                           np.maximum(1e-5 * np.abs(ref) + 4 * e32_all +
                                      np.broadcast_to(np.asarray(kink[k], np.float64), ref.shape), 1e-300)).max())
            print(f"step {s} {k}[{iw}]: ratio {rmax:.3g} (device err {dev_e:.3g}, ref {float(ref.flat[iw]):.3g}, "
                  f"E32 test {e32:.3g}); fp32 err at the element f32 {abs(g32[k].flat[iw] - ref.flat[iw]):.3g} "
                  f"f32r {abs(g32r[k].flat[iw] - ref.flat[iw]):.3g} relabelled "
                  f"[{', '.join(f'{e:.3g}' for e in el)}]; tensor max fp32 err relabelled "
                  f"[{', '.join(f'{e:.3g}' for e in tens)}]; ratio against the max over all {n_orders + 2} orders "
                  f"{r_all:.3g}", flush=True)


if __name__ == "__main__":
    main()
