"""HBM read rate of the data gradient's activation pattern (msat_probe_strip_read): the packed rows read as
register-A column strips (mode 0), as contiguous rows (1), as strips by three workgroups per row block (2).
usage: strip_probe.py [rows] [reps]"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import torch
from marlsat import _lib

P = _lib.probe_lib()
M = int(sys.argv[1]) if len(sys.argv) > 1 else 1316000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
H, K = 128, 384
torch.manual_seed(0)
D = torch.randn(M, 4 * H, device="cuda")
out = torch.empty(3 * ((M + 127) // 128) * 256, device="cuda")
s = _lib.stream_ptr()
for mode, name in ((0, "strips"), (1, "rows"), (2, "strips x3 workgroups")):
    for ptr, what in ((D.data_ptr(), "D[:, 0:3H]"), (D.data_ptr() + 4 * H, "D[:, H:4H]")):
        f = lambda: P.msat_probe_strip_read(ptr, M, 4 * H, K, mode, out.data_ptr(), s)
        for _ in range(2):
            assert f() == 0
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            f()
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) / reps * 1e3
        nb = 4.0 * M * K
        print(json.dumps({"pattern": name, "operand": what, "rows": M, "us": round(us, 1), "bytes": nb,
                          "GBps": round(nb / us / 1e3, 1)}), flush=True)
