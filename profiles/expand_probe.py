"""Two-phase env-step probe (diagnostic): price a grid-stride obs expansion from compact
bit images (per-env value bits, per-instance per-agent visibility bits) against the fused
kernel's per-workgroup chunked obs stores. uf200 shape: E=4096, A=25, D=2V+C=1260."""
import os, sys, statistics
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import torch
from marlsat import _lib
E, A, D, P = 4096, 25, 1260, 1024
Dw = (D + 31) // 32
g = torch.Generator(device="cuda").manual_seed(0)
def bits(n):
    return torch.randint(0, 2**31, (n,), device="cuda", dtype=torch.int64, generator=g).to(torch.int32)
inst = torch.randint(0, P, (E,), device="cuda", dtype=torch.int32, generator=g)
vimg, mimg = bits(E * Dw), bits(P * A * Dw)
out = torch.empty(E * A * D, dtype=torch.int32, device="cuda")
s = _lib.stream_ptr()
run = lambda grid: _lib.probe_lib().msat_probe_obs_expand(out.data_ptr(), E, A, D, inst.data_ptr(), vimg.data_ptr(),
                                                  mimg.data_ptr(), grid, s)
d = torch.arange(D, device="cuda")
for grid0 in (-4096, 4096):  # correctness on a sample of envs, both variants
  out.zero_()
  assert run(grid0) == 0
  torch.cuda.synchronize()
  for e in (0, 1, 777, E - 1):
    vb = (vimg.view(E, Dw)[e][d // 32].to(torch.int64) >> (d % 32)) & 1
    mb = (mimg.view(P, A, Dw)[inst[e].long()][:, d // 32].to(torch.int64) >> (d % 32)) & 1
    ref = torch.where(mb == 1, vb[None].expand(A, D), torch.full_like(mb, -1)).to(torch.int32)
    assert torch.equal(out.view(E, A, D)[e], ref), (grid0, e)
print("expand parity ok")
nbytes = E * A * D * 4
def t(grid, n=30):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for i in range(n):
        ev[i][0].record(); run(grid); ev[i][1].record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in ev) * 1e3
res = {}
for _ in range(2):
    for grid in (512, 1024, 2048, 4096, 8192, 16384, 32768, 65536, -512, -1024, -2048, -4096, -8192, -16384, -25600):
        res.setdefault(grid, []).append(t(grid))
for k, v in res.items():
    if isinstance(k, int):
        us = statistics.median(v)
        print(f"expand-{'rows' if k < 0 else 'quad'}-g{abs(k):<8d} {us:8.1f} us {nbytes/us/1e3:7.0f} GB/s")
