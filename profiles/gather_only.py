"""Clause gather (msat_clause_gather2: [A+^T H_v+ | A-^T H_v-], 3 signed slots per clause row) on the
uf50 training shape (1.036M clause rows from 407K var rows, H = 128), HIP-event timed, with its
algorithmic HBM rate (slots + 3 source rows read, one 2H row written per clause).
usage: gather_only.py [reps]
Measured 424 us (6.1 TB/s of slots + source rows + output); two rows per wave with the next slots
prefetched measured 431-446 us (bitwise equal output), not kept."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import torch
from marlsat import _lib

L = _lib.lib
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
H, Nv, Nc = 128, 407000, 1036000
s = _lib.stream_ptr()
g = torch.Generator(device="cuda").manual_seed(0)
Hp, Hn = torch.randn(Nv, H, device="cuda", generator=g), torch.randn(Nv, H, device="cuda", generator=g)
# each clause: 3 distinct-ish var rows, random signs (slot = (row << 1) | neg), clustered like a subgraph batch
base = torch.randint(0, Nv - 64, (Nc, 1), device="cuda", generator=g)
slots = ((base + torch.randint(0, 64, (Nc, 3), device="cuda", generator=g)) << 1 |
         torch.randint(0, 2, (Nc, 3), device="cuda", generator=g)).int().contiguous()
bwd = os.environ.get("GATHER_MODE") == "bwd"  # the backward's merged, accumulating form (dH_c += ...)
if bwd:
    Hp = torch.randn(Nv, 2 * H, device="cuda", generator=g)
    out = torch.zeros(Nc, H, device="cuda")
    f = lambda: L.msat_clause_gather2(Hp.data_ptr(), Hp.data_ptr() + 4 * H, 2 * H, slots.data_ptr(), out.data_ptr(),
                                      H, Nc, H, 1, 1, s)
else:
    out = torch.empty(Nc, 2 * H, device="cuda")
    f = lambda: L.msat_clause_gather2(Hp.data_ptr(), Hn.data_ptr(), H, slots.data_ptr(), out.data_ptr(), 2 * H, Nc,
                                      H, 0, 0, s)
assert f() == 0
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(reps):
    f()
b.record(); torch.cuda.synchronize()
us = a.elapsed_time(b) / reps * 1e3
# slots, 3 source rows of H floats read, one output row written (bwd: H wide, read and written)
nbytes = Nc * (12 + 3 * 4 * H + (8 * H if bwd else 8 * H))
print(json.dumps({"what": "clause_gather2" + (" bwd" if bwd else ""), "Nc": Nc, "us": round(us, 1), "GBps": round(nbytes / us / 1e3, 1),
                  "checksum": float(out.double().sum())}))
