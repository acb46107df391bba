"""Where does the fused step kernel's time go?  (diagnostic, run on the GPU box)

Interleaved rounds in ONE process (cdna_hip_programming.md §5.4 rule 24) of:
  full      — the product kernel
  constobs  — same kernel, obs pass replaced by constant 16 B stores (prices obs-value VALU/LDS work)
  noobs     — same kernel without the obs pass (prices the pre-obs phases)
  fill-nt / fill — a bare streaming store of the same obs bytes (the write ceiling)
"""
import os, sys, json, statistics
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import torch
from marlsat import SATEnv, _lib
from marlsat.random import Key
from marlsat.utils.generate_cnf_dataset import generate_problem_pool

wl = sys.argv[1] if len(sys.argv) > 1 else "uf200"
V, C, vpa, B = {"uf200": (200, 860, 8, 4096), "uf100": (100, 430, 10, 4096), "uf50": (50, 218, 10, 1024)}[wl]
env = SATEnv(V, C, max_steps=512, vars_per_agent=vpa)
pool = env.make_pool(generate_problem_pool(V, C, 256, size_id=3))
obs, st = env.reset_from_pool(pool, B, Key(1, 0))
out = env._step_out(B)
acts = torch.randint(0, env.max_vars_per_agent + 1, (16, B, env.num_agents), device="cuda", dtype=torch.int32)
step = env.stepper(st, obs, out, seed=5)
ctr = [1]

def time_steps(n=40):
    e = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for i in range(n):
        e[i][0].record(); step(acts[i % 16], ctr[0]); e[i][1].record(); ctr[0] += 1
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in e) * 1e3

def time_fill(nt, grid, n=40):
    nbytes = obs.numel() * obs.element_size()
    e = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    s = _lib.stream_ptr()
    for i in range(n):
        e[i][0].record(); _lib.probe_lib().msat_probe_fill(obs.data_ptr(), nbytes - nbytes % 16, -1, nt, grid, s); e[i][1].record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in e) * 1e3

res = {}
for rnd in range(3):
    for mode, name in ((0, "full"), (1, "constobs"), (2, "noobs"), (4, "full-noxcd")):
        os.environ["MARLSAT_ABLATE"] = str(mode)
        time_steps(5)
        res.setdefault(name, []).append(time_steps())
    os.environ["MARLSAT_ABLATE"] = "0"
    for nt in (1, 0):
        for grid in (1024, 4096, 16384):
            res.setdefault(f"fill{'-nt' if nt else ''}-g{grid}", []).append(time_fill(nt, grid))
obs_mb = obs.numel() * obs.element_size() / 1e6
summary = {k: {"us_median": statistics.median(v), "us_all": v} for k, v in res.items()}
for k, v in summary.items():
    v["obs_GBps"] = obs_mb * 1e3 / v["us_median"]
print(json.dumps({"workload": wl, "B": B, "obs_MB": obs_mb, "results": summary}, indent=1))
