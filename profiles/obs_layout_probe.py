"""Store-pattern probe for the env step's obs write (uf200 x 4096: 25 agents, D = 2V + C = 1,260 int32 = 315
x 16 B per row, 516 MB): one workgroup per env writes its 25 rows, env-major [E][A][D] (the product layout)
against agent-major [A][E][D] (each agent's rows of all envs contiguous), 256 / 512 lanes, grid = E or
capped (grid-stride over envs).  HIP events, reps launches per point.
usage: obs_layout_probe.py [reps]
Measured (profiles/r02_obs_layout_probe.log, two alternations): agent-major is 3-10 % SLOWER than env-major
at every point (best 121.4 vs 112.4 us), so the per-agent [A][E][D] obs layout was not pursued.  Per-row
loops with ragged tails (315 quads on 256 / 512 lanes) are themselves slower than the fused step kernel's
flat A*D image stores (108 us on the same bytes)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import torch
from marlsat import _lib

D = _lib.probe_lib()
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
E, A, D16 = 4096, 25, 315
buf = torch.empty(E * A * D16 * 4, dtype=torch.int32, device="cuda")
s = _lib.stream_ptr()
nbytes = buf.numel() * 4
for amajor in (0, 1, 0, 1):
    for threads in (256, 512):
        for grid in (E, 2048, 1024):
            f = lambda: D.msat_probe_fill_rows(buf.data_ptr(), E, A, D16, amajor, 7, threads, grid, s)
            assert f() == 0
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(reps):
                f()
            b.record()
            torch.cuda.synchronize()
            us = a.elapsed_time(b) / reps * 1e3
            print(json.dumps({"layout": "agent-major" if amajor else "env-major", "threads": threads, "grid": grid,
                              "us": round(us, 1), "GBps": round(nbytes / us / 1e3, 1)}), flush=True)
assert int(buf[::9973].min()) == 7
