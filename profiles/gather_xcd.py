"""Gathers on a graph batch shaped like the uf100-430 training micro-batch.  Per sample: the critic graph
(100 vars, 430 clauses) and 10 agent graphs (90 vars, 110 clauses each); every clause takes 3 distinct
signed var rows of its own graph, so source rows are shared only inside one graph, as in the real batch.
Times the four gather calls of one message-passing step (forward clause gather, forward var gather,
backward merged clause gather, backward var gather), HIP events, and prints a checksum per call.
usage: gather_xcd.py [samples] [reps]
Measured (profiles/r02_ab_gather_xcd.log, 820 samples: 1.25M clause rows, 0.82M var rows): 504-511 /
384-394 / 496-501 / 548-569 us.  An XCD-contiguous row walk (XCD x = blockIdx % 8 walks the contiguous
chunk x of the rows, so one graph's shared source rows stay in one L2) was built behind a switch and
measured against the grid-stride walk, alternating: 1955 / 1946 us against 1954 / 1952 us for the four
calls, i.e. neutral (the re-fetches across XCDs are served by the MALL), and removed.  Loading the next
row's slots while the current row's sources are in flight (one dependent round trip per row instead of
two) made the clause gathers 1-4 % slower (r02_ab_gather_pf.log: 493-501 vs 480-487 us): 32 resident
waves per CU already hide the chain.  PMC (profiles/ab_gather_walk.sh, r02_gather_walk/): with the XCD walk
each gather's L2 fabric reads fall to its minimal bytes (clause fwd 1.67 -> 0.81 GB, var fwd 1.81 -> 0.75,
clause bwd 2.31 -> 1.43, var bwd 2.74 -> 2.07) while the time stays within 1 % (grid cap 2048: -1 %,
1024: +42 %), so the gathers are bound by per-row latency at full occupancy, not by bytes."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import numpy as np
import torch
from marlsat import _lib

L = _lib.lib
S = int(sys.argv[1]) if len(sys.argv) > 1 else 820
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
H = 128
rng = np.random.default_rng(0)
graphs = [(100, 430)] + [(90, 110)] * 10
slot_rows, vbase = [], 0
for _ in range(S):
    for nv, nc in graphs:
        v = np.argsort(rng.random((nc, nv)), axis=1)[:, :3] + vbase
        slot_rows.append((v << 1) | rng.integers(0, 2, (nc, 3)))
        vbase += nv
slots_np = np.concatenate(slot_rows).astype(np.int32)
Nc, Nv = slots_np.shape[0], vbase
# var-side CSR: entries (clause_row << 1) | neg, ascending clause row per var
cl = np.repeat(np.arange(Nc), 3)
var = (slots_np >> 1).reshape(-1)
neg = (slots_np & 1).reshape(-1)
order = np.lexsort((cl, var))
inc_np = ((cl[order] << 1) | neg[order]).astype(np.int32)
ptr_np = np.zeros(Nv + 1, np.int64)
np.add.at(ptr_np, var + 1, 1)
ptr_np = np.cumsum(ptr_np).astype(np.int32)
dev = "cuda"
slots = torch.from_numpy(slots_np).to(dev)
inc, ptr = torch.from_numpy(inc_np).to(dev), torch.from_numpy(ptr_np).to(dev)
g = torch.Generator(device=dev).manual_seed(0)
Hp, Hn = torch.randn(Nv, H, device=dev, generator=g), torch.randn(Nv, H, device=dev, generator=g)
Hc = torch.randn(Nc, H, device=dev, generator=g)
GIN, NV = torch.empty(Nc, 2 * H, device=dev), torch.empty(Nv, 2 * H, device=dev)
dNV, dHc = torch.randn(Nv, 2 * H, device=dev, generator=g), torch.zeros(Nc, H, device=dev)
dGIN, dP, dN = torch.randn(Nc, 2 * H, device=dev, generator=g), torch.zeros(Nv, H, device=dev), torch.zeros(Nv, H, device=dev)
s = _lib.stream_ptr()
pp = lambda t, c=0: t.data_ptr() + 4 * c
calls = {
    "clause_fwd": lambda: L.msat_clause_gather2(pp(Hp), pp(Hn), H, pp(slots), pp(GIN), 2 * H, Nc, H, 0, 0, s),
    "var_fwd": lambda: L.msat_var_gather2(pp(Hc), pp(Hc), H, pp(ptr), pp(inc), pp(NV), pp(NV, H), 2 * H, Nv, H, 0, s),
    "clause_bwd": lambda: L.msat_clause_gather2(pp(dNV), pp(dNV, H), 2 * H, pp(slots), pp(dHc), H, Nc, H, 1, 1, s),
    "var_bwd": lambda: L.msat_var_gather2(pp(dGIN), pp(dGIN, H), 2 * H, pp(ptr), pp(inc), pp(dP), pp(dN), H, Nv, H,
                                          1, s),
}
nbytes = {  # slots / CSR + each source row once + output (read + written when accumulating)
    "clause_fwd": Nc * 12 + 2 * Nv * 4 * H + Nc * 8 * H,
    "var_fwd": Nv * 4 + Nc * 12 + Nc * 4 * H + Nv * 8 * H,
    "clause_bwd": Nc * 12 + Nv * 8 * H + Nc * 8 * H,
    "var_bwd": Nv * 4 + Nc * 12 + Nc * 8 * H + Nv * 16 * H,
}
out = {"samples": S, "Nc": Nc, "Nv": Nv}
for name, f in calls.items():
    assert f() == 0
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        f()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / reps * 1e3
    out[name] = {"us": round(us, 1), "GBps_min_bytes": round(nbytes[name] / us / 1e3, 1)}
# checksums of the non-accumulating outputs (identical for both walks: each row's sum order is fixed)
out["checksum"] = [float(GIN.double().sum()), float(NV.double().sum())]
print(json.dumps(out))
