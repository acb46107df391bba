"""The train-cycle test's bar applied to fixed-parameter gradients of several kernel paths (profiles/parity_attrib.py
output) on the CPU: float64 oracle, the fp32 oracle in two row orders (E32) and the ReLU-kink allowance as in
tests/test_mappo_gpu.py; prints, per path, the worst ratio to the bar and its tensor.

    python profiles/parity_compare.py <dump.npz> <step> <attrib.npz>
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "marl-sat_amd"), os.path.join(ROOT, "profiles")):
    sys.path.insert(0, p)

from marlsat.learners import params as Pm  # noqa: E402
import parity_orderings as po  # noqa: E402


def main():
    path, s, apath = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    d = np.load(path)
    V, C, vpa, H, L, mode, T, B, MB, E = (int(v) for v in d["shape"])
    A, M = d["av"].shape
    cfg = po.cfg_of(d["shape"])
    av, am = torch.from_numpy(d["av"].astype(np.int64)), torch.from_numpy(d["am"])
    full = {k[5:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("full_")}
    mb = {k: v[d[f"idx_{s}"]] for k, v in full.items()}
    P = Pm.to_flax(d[f"params_{s}"].astype(np.float32), H, L, A, M, mode, 16)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    g64, kink = po.grads(P, mb, cfg, av, am, mode, L, torch.float64, log=True)
    g32, _ = po.grads(P, mb, cfg, av, am, mode, L, torch.float32)
    rows = torch.from_numpy(np.arange(len(d[f"idx_{s}"]))[::-1].copy())
    g32r, _ = po.grads(P, {k: v[rows] for k, v in mb.items()}, cfg, av, am, mode, L, torch.float32)
    a = np.load(apath)
    for lab in a.files:
        t = Pm.to_flax(a[lab], H, L, A, M, mode, 16)
        ratios = []
        for k in g64:
            ref = g64[k]
            e32 = max(np.abs(g32[k] - ref).max(), np.abs(g32r[k] - ref).max())
            kb = np.broadcast_to(np.asarray(kink[k], np.float64), ref.shape)
            r = (np.abs(np.asarray(t[k], np.float64) - ref) / np.maximum(1e-5 * np.abs(ref) + 4 * e32 + kb, 1e-300)).max()
            ratios.append((float(r), k))
        ratios.sort(reverse=True)
        print(f"{os.path.basename(path)} step {s} {lab}: worst ratio {ratios[0][0]:.3g} ({ratios[0][1]}); next "
              + ", ".join(f"{k} {r:.3g}" for r, k in ratios[1:3]), flush=True)


if __name__ == "__main__":
    main()
