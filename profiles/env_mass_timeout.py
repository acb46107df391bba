"""Per-launch time of the auto-reset env step from a fresh reset (every episode counter at 0), so that the whole
batch times out together at launch 511 (and again at 1023): the launches around those, against the median, with
the reset queue on or off (MARLSAT_RESET_QUEUE).  One HIP event pair per launch.

    python profiles/env_mass_timeout.py [workload envs]      (default uf50-218 1024)
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from marlsat import SATEnv  # noqa: E402
from marlsat.random import Key  # noqa: E402
from marlsat.utils.generate_cnf_dataset import generate_problem_pool  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "uf50-218"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
V, C, vpa, _, sid = bench.WORKLOADS[wl]
env = SATEnv(V, C, max_steps=512, vars_per_agent=vpa)
pool = env.make_pool(generate_problem_pool(V, C, 256, size_id=sid))
obs, st = env.reset_from_pool(pool, B, Key(7, 0))
out = env._step_out(B)
step = env.stepper(st, obs, out, autoreset=True, seed=7)
g = torch.Generator(device="cuda").manual_seed(0)
acts = torch.randint(0, env.max_vars_per_agent + 1, (64, B, env.num_agents), generator=g, device="cuda", dtype=torch.int32)
N = 1100
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(N)]
for i in range(N):
    ev[i][0].record()
    step(acts[i % 64], i + 1)
    ev[i][1].record()
torch.cuda.synchronize()
t = [a.elapsed_time(b) * 1e3 for a, b in ev]
med = statistics.median(t[20:])
print(f"{wl} x {B}, queue {os.environ.get('MARLSAT_RESET_QUEUE', '1')}: median {med:.2f} us; launches 509-513: "
      f"{[round(x, 1) for x in t[509:514]]}; 1021-1025: {[round(x, 1) for x in t[1021:1026]]}; "
      f"max outside them {max(x for i, x in enumerate(t[20:], 20) if not (509 <= i <= 513 or 1021 <= i <= 1025)):.1f} us")
