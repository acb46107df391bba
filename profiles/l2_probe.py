"""Texture-path probe (msat_probe_l2_read): L2-resident reads at the data gradient's occupancy, as plain loads
and as LDS-DMA pieces, lane-linear and in the kernels' own patterns; GB/s per CU.  usage: l2_probe.py [iters] [reps]"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import torch
from marlsat import _lib

P = _lib.probe_lib()
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
cus = torch.cuda.get_device_properties(0).multi_processor_count
grid = 3 * cus
window = 2 << 20
buf = torch.randn(window // 4 + 65536, device="cuda")
out = torch.empty(grid * 256, device="cuda")
s = _lib.stream_ptr()
names = {0: "loads, lane-linear", 1: "LDS-DMA, lane-linear", 2: "loads, register-A pattern (16 rows x 4 x 16 B at 32 B)",
         3: "LDS-DMA, weight-piece pattern (16 rows x 64 B)", 4: "loads, 8 rows x 128 B", 5: "loads, 16 rows x 64 B"}
cases = [(0, 0), (1, 0), (3, 768), (3, 2048)] + [(m, st) for m in (2, 4, 5) for st in (2048, 2048 + 128, 768)]
for mode, stride in cases:
    f = lambda: P.msat_probe_l2_read(buf.data_ptr(), window, mode, iters, grid, max(stride, 128), out.data_ptr(), s)
    assert f() == 0
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        f()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / reps * 1e3
    nb = float(grid) * 4 * iters * 1024
    print(json.dumps({"mode": mode, "form": names[mode], "row_stride_B": stride, "us": round(us, 1), "GBps": round(nb / us / 1e3, 1),
                      "GBps_per_CU": round(nb / us / 1e3 / cus, 2)}), flush=True)
