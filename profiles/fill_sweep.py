"""HBM write-pattern sweep (diagnostic): grid-stride vs per-block-contiguous 16 B stores."""
import os, sys, json, statistics
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import torch
from marlsat import _lib
nbytes = 4096 * 25 * 1260 * 4
buf = torch.empty(nbytes // 4, dtype=torch.int32, device="cuda")
s = _lib.stream_ptr()
def t(fn, nt, grid, n=30):
    e = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for i in range(n):
        e[i][0].record(); fn(buf.data_ptr(), nbytes, -1, nt, grid, s); e[i][1].record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in e) * 1e3
res = {}
for rnd in range(2):
    for name, fn in (("stride", _lib.probe_lib().msat_probe_fill), ("chunk", _lib.probe_lib().msat_probe_fill_chunked)):
        for nt in (0, 1):
            for grid in (512, 1024, 2048, 4096, 8192, 16384, 32768, 65536):
                res.setdefault(f"{name}-nt{nt}-g{grid}", []).append(t(fn, nt, grid))
for k, v in res.items():
    us = statistics.median(v)
    print(f"{k:24s} {us:8.1f} us {nbytes/us/1e3:7.0f} GB/s")
