"""Headline benchmark: batched SATEnv.step (+ rollout auto-reset) env-steps/sec.

Workload (BASELINE.json configs[3], one GPU's shard): uf200-860 random 3-SAT,
VARS_PER_AGENT=8 -> 25 agents, 4096 envs per GPU, MAX_STEPS=512, auto-reset on
(done envs redraw a pool instance + a Bernoulli(0.5) assignment on the device),
mode-0 actions uniform over [0, M] pre-generated on the device (outside the
timed region), obs int32 (the reference dtype).  One "step" = one fused
``msat_env_step`` launch over the whole local batch.

Multi-GPU (torchrun, one process per GPU): independent env shards, no
collective on the data path; barrier + synchronize around the timed region,
max elapsed over ranks; value = all ranks' env-steps / that time (weak scaling).
``python bench.py --gpus N`` without torchrun's env times the CPU baselines and
then starts ``python -m torch.distributed.run --nproc-per-node N bench.py ...``
as a child process; a world size that disagrees with ``--gpus`` fails.

MAPPO legs (the metric's "MAPPO updates/sec"): one full train cycle of the device
learner -- rollout of T steps (actor + critic forward, sampling, fused env step with
auto-reset), GAE + global advantage normalisation, UPDATE_EPOCHS x T*B/MINIBATCH_SIZE
PPO minibatches (forward, loss, backward, gradient all-reduce over RCCL when N>1,
Adam) and the cycle metrics -- timed after one warm-up cycle.  The headline leg is
uf100-430 x 4096 envs (BASELINE config 3, the metric's 4096 envs), T = 8; uf200-860 x
4096 envs per GPU, 25 agents, T = 2 (config 4) is reported beside it.  Each leg carries
per-phase times and its roofline: the dominant matrix kernel (HIP events around each launch,
algorithmic FLOPs and HBM bytes per launch) against the lower of its two roofs, the ceiling of
the matrix instruction it issues (fp16 dense / 3 for the fp16x2 kernels, bf16 dense / 6 for
bf16x3) and its intensity x the 8 TB/s HBM peak.  The full per-kernel tables go to a side
file under gpurun_out/.

Prints ONE JSON line on rank 0; the MAPPO legs close it.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import socket
import statistics
import subprocess
import sys
import time
from typing import Optional

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "marl-sat_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "env-steps/sec (whole node) + MAPPO updates/sec, 4096 envs random 3-SAT"
WORKLOADS = {  # name: V, C, vars_per_agent, envs per GPU, size_id (seed = 1000*size_id + i)
    "uf20-91": (20, 91, 10, 8, 0),
    "uf50-218": (50, 218, 10, 1024, 1),
    "uf100-430": (100, 430, 10, 4096, 2),
    "uf200-860": (200, 860, 8, 4096, 3),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X dense fp32 matrix peak (MI355X_MICROARCH.md)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 matrix peak (~2.5 PF, MI355X_MICROARCH.md)
# the bf16x3 kernels issue 6 bf16 MFMAs per fp32 product (x1y1, x1y2, x2y1, x1y3, x2y2, x3y1):
# their ceiling in fp32-equivalent FLOP/s is the bf16 dense peak / 6
X3_PEAK_TFLOPS = BF16_MFMA_PEAK_TFLOPS / 6.0



def env_lanes(A: int, D: int, B: int) -> int:
    """Workgroup size the env step launches with (env_kernels.hip env_threads): for the kernel label."""
    n = A * D
    if n >= 16384:
        return 512
    if n > 4096:
        return 256 if B <= 1024 else 128
    return 128 if B <= 1024 else 64

def step_bytes(V: int, C: int, A: int) -> int:
    """Algorithmic bytes of one env-step (reference API dtypes)."""
    D = 2 * V + C
    bytes_in = 12 * C + 4 * V + 4 + 4 * A
    bytes_out = 4 * A * D + 4 * V + C + 4 + 4 + A + 4 * A + (A + 1) + 9
    return bytes_in + bytes_out


# ------------------------------------------------------------ CPU baseline ----
def _cpu_worker(args):
    V, C, vpa, nenv, budget, wid, pool = args
    import numpy as np
    from threadpoolctl import threadpool_limits

    from oracle.sat_env import OracleSATEnv

    with threadpool_limits(1):
        rng = np.random.default_rng(wid)
        env = OracleSATEnv(V, C, max_steps=512, vars_per_agent=vpa)
        N = pool.shape[0]
        _, st = env.reset(pool[rng.integers(0, N, nenv)], rng.integers(0, 2, (nenv, V)))
        M = env.max_vars_per_agent
        steps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < budget:
            a = rng.integers(0, M + 1, (nenv, env.num_agents))
            newp = pool[rng.integers(0, N, nenv)]
            newx = rng.integers(0, 2, (nenv, V))
            _, st, _, _, _ = env.step_autoreset(st, a, newp, newx)
            steps += 1
        return steps * nenv, time.perf_counter() - t0


def host_cpu() -> dict:
    """The host the CPU baselines run on: model name (/proc/cpuinfo, as lscpu prints it), the cores
    this process may run on (sched_getaffinity) and the cores used: min(affinity, the cgroup's CPU quota,
    the cap).  The cap is OMP_NUM_THREADS (16 per GPU on the GPU pool, where the affinity mask shows the
    whole machine but the cgroup allows 16 CPUs); MARLSAT_CPU_BASELINE_CORES overrides it."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    cap_src = "MARLSAT_CPU_BASELINE_CORES" if os.environ.get("MARLSAT_CPU_BASELINE_CORES") else (
        "OMP_NUM_THREADS" if os.environ.get("OMP_NUM_THREADS") else "affinity")
    cap = int(os.environ.get("MARLSAT_CPU_BASELINE_CORES") or os.environ.get("OMP_NUM_THREADS") or affinity)
    quota = cgroup_cpus()
    cores = min(affinity, cap)
    if quota:  # more processes than the quota only time-share it
        if int(quota) < cores:
            cap_src = "cgroup quota"
        cores = min(cores, int(quota))
    return {"cpu_model": model, "affinity_cores": affinity, "cores": max(1, cores),
            "cap_source": cap_src, "cgroup_cpus": quota}


def cgroup_cpus():
    """The CPU time this process's cgroup may use, in CPUs (cgroup v2 cpu.max quota / period; v1
    cfs_quota / cfs_period), or None when unlimited or unreadable: a process pool larger than this
    shares that much CPU, whatever the affinity mask shows."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return None if q <= 0 else round(q / per, 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(V, C, vpa, pool, budget_s=12.0, nenv=16, cores=None):
    """Reference algorithm restated in NumPy (oracle), one single-thread process per host core
    (``cores`` processes; default: the box's CPU share, host_cpu())."""
    import multiprocessing as mp

    host = host_cpu()
    procs = host["cores"] if cores is None else cores
    ctx = mp.get_context("fork")  # forked before any GPU initialisation
    with ctx.Pool(procs) as p:
        res = p.map(_cpu_worker, [(V, C, vpa, nenv, budget_s, w, pool) for w in range(procs)])
    total = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    # cores = CPUs the processes actually had: never more than the cgroup quota, however many processes ran
    used = min(procs, host["cores"]) if cores is None else min(procs, int(host["cgroup_cpus"] or procs))
    over = procs > used
    return {
        "value": total / wall,
        "unit": "env-steps/s",
        "cores": used,
        "processes": procs,
        "oversubscribed": over,
        "kind": "port",
        "host": host,
        "sample": f"oracle/sat_env.py step_autoreset (reference algorithm: full rescan, dense int32 obs, "
                  f"reset-all-then-select) on {procs} single-thread processes x {nenv} envs of the same workload, "
                  f"{budget_s:.0f} s each ({total} env-steps); host {host['cpu_model']}, "
                  f"{host['affinity_cores']} cores in the affinity mask, cgroup quota {host['cgroup_cpus']} CPUs, "
                  f"{used} CPUs used ({host['cap_source'] if cores is None else 'explicit process count'})"
                  + (f"; OVERSUBSCRIBED: {procs} processes time-share {used} CPUs" if over else ""),
    }


# ------------------------------------------------------------------- PMC ----
def _round_of(path: str) -> int:
    """The round a committed profile belongs to, from its path (profiles/r05/..., profiles/r04_pmc.json)."""
    import re

    tags = re.findall(r"(?:^|[/_])r(\d\d)", os.path.relpath(path, ROOT))
    return max((int(t) for t in tags), default=0)


def load_pmc_traffic(workload: str, kernel: str, default_shape: bool = True):
    """HBM bytes per launch of the step kernel from the newest committed rocprofv3 PMC summary under
    profiles/ (any depth, archives excluded): either {"workload", "hbm_bytes_per_launch"} records
    (profiles/collect.sh) or per-kernel tables {kernel: {"per_launch_bytes": {"total"}}}
    (profiles/pmc_env_summary.py), matched on the kernel instantiation the leg launches; a table without a
    "workload" key was collected on the bench's default legs, so it serves only default_shape runs."""
    files = [f for f in glob.glob(os.path.join(ROOT, "profiles", "**", "*pmc*.json"), recursive=True)
             if "archive" not in f]
    files.sort(key=lambda f: (_round_of(f), f))
    want = kernel.replace(" ", "")
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if not isinstance(d, dict):
            continue
        if d.get("workload") == workload and d.get("hbm_bytes_per_launch"):
            return float(d["hbm_bytes_per_launch"]), os.path.relpath(f, ROOT)
        if d.get("workload", workload if default_shape else None) != workload:
            continue
        for k, v in d.items():
            if isinstance(v, dict) and k.replace(" ", "") == want and (v.get("per_launch_bytes") or {}).get("total"):
                return float(v["per_launch_bytes"]["total"]), os.path.relpath(f, ROOT)
    return None, None


def load_gru_pmc_ratio():
    """PMC HBM bytes / algorithmic bytes of the GRU forward (the newest profiles/*pmc_gru.json: FETCH_SIZE x 2 +
    WRITE_SIZE per launch on the clause and var training shapes, profiles/pmc_gru_traffic.sh)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_gru.json")))
    if not files:
        return None, None
    f = files[-1]
    try:
        d = json.load(open(f))
        r = [v["pmc_over_algorithmic"] for v in d.values()]
        return sum(r) / len(r), os.path.basename(f)
    except Exception:
        return None, None


# ------------------------------------------------------------------ MAPPO ----
def mappo_cpu_baseline(workload: str, budget_s: float = 10.0, batch: int = 8):
    """PPO minibatch forward + backward of the reference network restated in torch (oracle/net.py:
    dense masked per-agent encoders, as the reference computes them), float32, all host cores
    (<= 16), on the MAPPO leg's instance size: samples/s over ~budget_s."""
    import numpy as np
    import torch

    from marlsat.utils.generate_cnf_dataset import generate_problem_pool
    from oracle import net as onet
    from oracle.sat_env import OracleSATEnv

    host = host_cpu()
    cores = host["cores"]
    prev = torch.get_num_threads()
    torch.set_num_threads(cores)
    try:
        V, C, vpa, _, size_id = WORKLOADS[workload]
        pool = generate_problem_pool(V, C, batch, size_id=size_id)
        ora = OracleSATEnv(V, C, 512, vars_per_agent=vpa)
        A, M = ora.num_agents, ora.max_vars_per_agent
        rng = np.random.default_rng(0)
        x = rng.integers(0, 2, (batch, V)).astype(np.int32)
        _, st = ora.reset(pool, x)
        Ap, An = onet.dense_graph(pool, V)
        f32 = lambda a: torch.as_tensor(np.asarray(a), dtype=torch.float32)
        mb = {"svf": f32(ora.static_var_features(pool)), "x": f32(x), "cf": f32(ora.clause_features(st)),
              "A_pos": Ap.float(), "A_neg": An.float(), "action": torch.from_numpy(rng.integers(0, M + 1, (batch, A))),
              "log_prob": f32(rng.normal(-1.5, 0.3, (batch, A))), "value": f32(rng.normal(0, 0.5, batch)),
              "targets": f32(rng.normal(0, 1, batch)), "gae": f32(rng.normal(0, 1, batch))}
        P = onet.init_params(onet.param_shapes(128, 16, A, M, 0), seed=0, dtype=torch.float32)
        av, am = torch.from_numpy(ora.agent_vars.astype(np.int64)), torch.from_numpy(ora.action_mask)
        cfg = {"CLIP_EPS": 0.2, "VF_CLIP": 0.2, "ENT_COEF": 0.01, "VF_COEF": 0.5}
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < budget_s:
            Pk = {k: v.clone().requires_grad_(True) for k, v in P.items()}
            total, _, _, _ = onet.ppo_loss(Pk, 16, mb, cfg, av, am, 0)
            total.backward()
            n += batch
        wall = time.perf_counter() - t0
    finally:
        torch.set_num_threads(prev)
    return {"value": n / wall, "unit": "PPO samples/s (minibatch forward + backward)", "cores": cores,
            "kind": "port", "host": host,
            "sample": f"oracle/net.py ppo_loss + autograd (reference GNN_ActorCritic restated: dense masked per-agent "
                      f"encoders), float32, {workload}, H=128, L=16, minibatches of {batch}, {n} samples in {wall:.1f} s; "
                      f"host {host['cpu_model']}, {cores} torch threads of {host['affinity_cores']} affinity cores"}


def kernel_table(ktimer: dict) -> list:
    """Per-kernel totals of the GNN's MFMA launches recorded by GNNActorCritic.ktimer (HIP events on
    the launch stream around each launch): average duration and fp32-equivalent TFLOP/s against the
    ceiling of the instruction the kernel issues (bf16 dense / 6 for the bf16x3 kernels, fp32 MFMA
    for the fp32 ones).  Sorted by total time."""
    rows = []
    for label, recs in ktimer.items():
        ms = sum(a.elapsed_time(b) for a, b, _, _ in recs)
        fl = sum(f for _, _, f, _ in recs)
        nb = sum(n for _, _, _, n in recs)
        if "K <= 8" in label:
            peak, unit_note = None, "HBM-bound (K <= 8 columns), not priced against a matrix peak"
        elif "fp16x2" in label:
            peak, unit_note = BF16_MFMA_PEAK_TFLOPS / 3.0, "fp16 dense peak (= bf16) / 3 (three fp16 MFMAs per fp32 product)"
        elif "bf16x3" in label:
            peak, unit_note = X3_PEAK_TFLOPS, "bf16 dense peak / 6 (six bf16 MFMAs per fp32 product)"
        else:
            peak, unit_note = FP32_MFMA_PEAK_TFLOPS, "fp32 MFMA peak"
        tf = fl / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
        gbs = nb / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        row = {"kernel": label, "launches": len(recs), "ms_total": ms, "ms_avg": ms / len(recs),
               "tflops_fp32_equiv": tf, "peak": peak, "frac": (tf / peak) if peak else None,
               "peak_basis": unit_note, "algorithmic_bytes_avg": nb / len(recs), "hbm_GBps": gbs,
               "hbm_frac": gbs / HBM_PEAK_GBS}
        if peak and nb > 0:
            # roofline: attainable = min(matrix ceiling, intensity x HBM peak); frac against the lower roof
            inten = fl / nb  # fp32-equivalent FLOP per algorithmic byte
            roof = min(peak, inten * HBM_PEAK_GBS / 1e3)
            row.update({"intensity_flop_per_byte": inten, "bound": "mfma" if peak <= roof + 1e-9 else "hbm",
                        "attainable_tflops": roof, "roofline_frac": tf / roof})
        rows.append(row)
    rows.sort(key=lambda r: -r["ms_total"])
    return rows


def mappo_roofline(dom: dict, workload: str) -> dict:
    """The MAPPO leg's roofline object for its dominant matrix kernel: against the lower of its two roofs
    (the matrix ceiling of the instruction it issues, and its algorithmic intensity x the HBM peak).
    HBM-bound: achieved = algorithmic GB/s vs 8 TB/s; MFMA-bound: fp32-equivalent TF/s vs the ceiling.
    Both views are carried either way."""
    hbm = dom.get("bound") == "hbm"
    ratio, src = load_gru_pmc_ratio() if "gru_ln_fused_fwd_h2s" in dom["kernel"] else (None, None)
    alg = dom.get("algorithmic_bytes_avg")
    r = {"bound": "hbm" if hbm else "mfma", "kernel": dom["kernel"],
         "achieved": dom["hbm_GBps"] if hbm else dom["tflops_fp32_equiv"],
         "peak": HBM_PEAK_GBS if hbm else dom["peak"], "unit": "GB/s" if hbm else "TFLOP/s (fp32-equivalent)",
         "frac": dom["hbm_frac"] if hbm else dom["frac"],
         "traffic": ratio * alg if ratio and alg else None,
         "traffic_source": (f"{src}: PMC bytes = {ratio:.3f} x algorithmic on the clause / var training shapes"
                            if ratio else None),
         "kernel_ms": dom["ms_avg"], "launches": dom["launches"],
         "algorithmic_bytes_per_launch": dom.get("algorithmic_bytes_avg"),
         "mfma": {"achieved_tflops_fp32_equiv": dom["tflops_fp32_equiv"], "peak": dom["peak"], "frac": dom["frac"]},
         "hbm": {"achieved_GBps": dom["hbm_GBps"], "peak": HBM_PEAK_GBS, "frac": dom["hbm_frac"]},
         "intensity_flop_per_byte": dom.get("intensity_flop_per_byte"),
         "frac_of_attainable": dom.get("roofline_frac"),
         "note": f"dominant matrix kernel of the timed cycle, algorithmic FLOPs / bytes over its HIP-event time "
                 f"(DESIGN.md §7); rocprof slice: profiles/*_mappo_{workload}_slice.json"}
    return r


def progress(rank: int, msg: str) -> None:
    """A line on stderr per bench phase (rank 0): long silent stretches (the MAPPO legs run minutes without
    output) are otherwise indistinguishable from a hang to a watchdog; stdout keeps only the JSON line."""
    if rank == 0:
        print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _timed_cycle(learner, rs, gen, dist):
    """One MAPPO train cycle from runner state rs, phase by phase: (wall s, [rollout, gae, ppo_update, metrics]
    ms, metrics, the new runner state)."""
    import torch

    ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev[0].record()
    rs = learner.rollout(rs)
    ev[1].record()
    learner.compute_advantages(rs)
    ev[2].record()
    losses, ent = learner.ppo_update(1, gen)
    ev[3].record()
    met = learner.metrics(losses, ent)
    ev[4].record()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    return time.perf_counter() - t0, [ev[i].elapsed_time(ev[i + 1]) for i in range(4)], met, rs


def _max_over_ranks(cycles, dist):
    """The slowest rank's wall time and phases, per cycle."""
    import torch

    if dist is None:
        return cycles
    t = torch.tensor([v for c in cycles for v in [c[0]] + c[1]], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [(r[0], r[1:]) for r in t.view(len(cycles), 5).tolist()]


def mappo_bench(args, rank, world, dist, workload: str, B: int, T: int, fp32_cycles: int = 0):
    """Timed MAPPO train cycles (after one warm-up cycle) on the stated config; with fp32_cycles, that many
    more cycles on the fp32 path (MARLSAT_PRECISION=fp32: fp32 MFMA in the reference's operation order) of the
    same learner, reported beside the default path's time."""
    import torch

    from marlsat import SATEnv
    from marlsat.learners.gnn import GNNActorCritic
    from marlsat.learners.mappo_gnn_sat_learner import MAPPOLearner
    from marlsat.random import PRNGKey
    from marlsat.utils.generate_cnf_dataset import generate_problem_pool

    V, C, vpa, _, size_id = WORKLOADS[workload]
    E = 4
    H, L = 128, 16
    cfg = dict(NUM_ENVS=B, NUM_STEPS=T, UPDATE_EPOCHS=E, MINIBATCH_SIZE=B * T // 4, NUM_UPDATES=1000,
               LEARNING_RATE=3e-4, ANNEAL_LR=True, LR_START_FACTOR=1.0, LR_END_FLOOR=1e-5, GAMMA=0.99,
               GAE_LAMBDA=0.95, CLIP_EPS=0.2, ENT_COEF=0.01, VF_COEF=0.5, VF_CLIP=0.2,
               GNN_HIDDEN_DIM=H, GNN_NUM_MESSAGE_PASSING_STEPS=L, action_mode=0,
               MICROBATCH_BYTES=args.mappo_micro_gb * 1e9)
    env = SATEnv(V, C, max_steps=512, vars_per_agent=vpa)
    # instances leaving a variable in no clause are skipped: at zero-initialised biases that variable is a
    # constant LayerNorm row whose gradient overflows fp32 in the reference too (generate_problem_pool doc)
    pool = env.make_pool(generate_problem_pool(V, C, args.pool, size_id=size_id, skip_isolated=True))
    net = GNNActorCritic(H, L, env.num_agents, env.max_vars_per_agent, 0, V, device=env.device, seed=0)
    comm = dist if world > 1 else None
    if comm is not None and os.environ.get("MARLSAT_COLLECTIVES") == "capi":
        # the learner's all-reduces through the C-ABI communicator (msat_comm_init / msat_allreduce_sum)
        from marlsat.learners.collectives import CapiComm

        comm = CapiComm.from_dist(dist)
    learner = MAPPOLearner(cfg, env, net, pool, dist=comm)
    rs = learner.init_runner_state(PRNGKey(77 + rank))
    gen = torch.Generator().manual_seed(99 + rank)
    progress(rank, f"mappo {workload} x {B}, T {T}: warm-up")
    learner.cfg["UPDATE_EPOCHS"] = 1  # warm-up cycle (every kernel and buffer shape), one epoch
    rs, _ = learner.train_cycle(rs, 0, gen)
    progress(rank, f"mappo {workload}: {args.mappo_cycles} timed cycles")
    learner.cfg["UPDATE_EPOCHS"] = E
    torch.cuda.synchronize()
    GNNActorCritic.flops = 0
    GNNActorCritic.ktimer = {}  # per-launch HIP events over every timed cycle
    cycles = []  # (wall s, [rollout, gae, ppo_update, metrics] ms) per timed cycle
    for _ in range(args.mappo_cycles):
        wall, ph, met, rs = _timed_cycle(learner, rs, gen, dist)
        cycles.append((wall, ph))
    flops = float(GNNActorCritic.flops) / len(cycles)
    kernels = kernel_table(GNNActorCritic.ktimer)
    GNNActorCritic.ktimer = None
    dom = next(k for k in kernels if k["peak"])  # the matrix kernel with the most time in the cycles
    rank_ms = [0.0] * world  # each rank's dominant-kernel average launch time
    rank_ms[rank] = dom["ms_avg"]
    cycles = _max_over_ranks(cycles, dist)
    per_cycle = [c[0] for c in cycles]
    if dist is not None:
        rk = torch.tensor(rank_ms, dtype=torch.float64, device="cuda")
        dist.all_reduce(rk)  # every rank fills its own slot: SUM = gather
        rank_ms = [float(v) for v in rk]
    elapsed = statistics.median(per_cycle)
    phases = [statistics.median(c[1][i] for c in cycles) for i in range(4)]
    cycle_ms = sum(sum(c[1]) for c in cycles)
    fp32 = None
    if fp32_cycles:  # the same learner on the fp32 path: what the split arithmetic buys (BASELINE.md:57)
        from marlsat.learners import gnn as gnn_mod

        progress(rank, f"mappo {workload}: {fp32_cycles} fp32-path cycle(s)")
        prev = gnn_mod.set_precision("fp32")
        try:
            c32 = []
            for _ in range(fp32_cycles):
                wall, ph, _, rs = _timed_cycle(learner, rs, gen, dist)
                c32.append((wall, ph))
            c32 = _max_over_ranks(c32, dist)
        finally:
            gnn_mod.restore_precision(prev)
        s32 = statistics.median(c[0] for c in c32)
        fp32 = {"s_per_update": s32, "s_per_update_cycles": [c[0] for c in c32],
                "phase_ms": dict(zip(("rollout", "gae", "ppo_update", "metrics"),
                                     [statistics.median(c[1][i] for c in c32) for i in range(4)])),
                "speedup_of_default": s32 / elapsed,
                "note": "MARLSAT_PRECISION=fp32 (fp32 MFMA throughout, phi not folded: the reference's operation "
                        "order), same learner and config, timed after the default path's cycles (no extra warm-up)"}
    replicas = replica_check(net, dist)
    if type(comm).__name__ == "CapiComm":
        comm.destroy()
    n_mb = B * T // cfg["MINIBATCH_SIZE"]
    gemm_tflops = flops / (elapsed * 1e12)
    for k in kernels:
        k["share_of_cycle"] = k["ms_total"] / cycle_ms
    roof = mappo_roofline(dom, workload)
    roof["per_rank_kernel_ms"] = rank_ms
    full = {
        "metric": "MAPPO updates/sec",
        "value": 1.0 / elapsed,
        "unit": "updates/s",
        "s_per_update": elapsed,
        "s_per_update_cycles": per_cycle,
        "adam_steps_per_s": E * n_mb / elapsed,
        "samples_per_s": world * B * T / elapsed,
        "ppo_samples_per_s": world * E * B * T / (phases[2] * 1e-3),
        "phase_ms": dict(zip(("rollout", "gae", "ppo_update", "metrics"), phases)),
        "config": {"workload": workload, "num_agents": env.num_agents, "max_vars_per_agent": env.max_vars_per_agent,
                   "envs_per_gpu": B, "global_envs": B * world, "NUM_STEPS": T, "UPDATE_EPOCHS": E,
                   "MINIBATCH_SIZE": cfg["MINIBATCH_SIZE"], "GNN_HIDDEN_DIM": H, "GNN_NUM_MESSAGE_PASSING_STEPS": L,
                   "micro_batch": learner.micro,
                   "pool": f"{args.pool} instances, seeds 1000*{size_id}+i, instances with an unused variable skipped",
                   "parallelism": f"dp{world} (env shards; RCCL gradient all-reduce per minibatch"
                                  f"{', C-ABI communicator' if type(comm).__name__ == 'CapiComm' else ''})"},
        "roofline": roof,
        "kernels": kernels,
        "issued_gemm_tflops_over_cycle": gemm_tflops,
        "dtype": "f32 (fp32 accumulate; fp16x2 split MFMAs, bf16x3 where fp16's range does not hold)",
        "solve_rate": met["solve_rate"],
        "params_check": replicas,
        "peak_hbm_gb": torch.cuda.max_memory_allocated() / 1e9,
        "fp32_path": fp32,
    }
    side = write_side_file(f"mappo_{workload}_n{world}_rank{rank}", full)
    return compact_leg(full, side)


def _sig(x, n=4):
    return float(f"{x:.{n}g}") if isinstance(x, float) else x


def compact_leg(full: dict, side: Optional[str]) -> dict:
    """The MAPPO leg as it goes into the JSON line: ~0.6 KB, so the env side legs and both MAPPO legs fit the
    driver's 2,000-character tail (which also holds the run's stderr).  value = 1 / the median of the timed
    cycles' s_per_update (with --mappo-cycles 3, the default, a true median of three).  The full record (per-kernel table, both roofline views) is in the side file."""
    c, r = full["config"], full["roofline"]
    ph = full["phase_ms"]
    cyc = full.get("s_per_update_cycles", [full["s_per_update"]])
    out = {
        "value": _sig(full["value"]),
        # min / median / max over the timed cycles (each cycle's time, in order, and Adam steps/s: side file)
        "s_min_med_max": [_sig(min(cyc)), _sig(full["s_per_update"]), _sig(max(cyc))],
        "samples_per_s": _sig(full["samples_per_s"]),
        "phase_ms": [round(ph[k]) for k in ("rollout", "gae", "ppo_update", "metrics")],
        "config": f"{c['workload']} A{c['num_agents']} m{c['max_vars_per_agent']} B{c['envs_per_gpu']}/gpu "
                  f"T{c['NUM_STEPS']} E{c['UPDATE_EPOCHS']} mb{c['MINIBATCH_SIZE']} H{c['GNN_HIDDEN_DIM']} "
                  f"L{c['GNN_NUM_MESSAGE_PASSING_STEPS']} {c['parallelism'].split(' ')[0]}",
        "roofline": {"bound": r["bound"], "achieved": _sig(r["achieved"]), "peak": r["peak"],
                     "unit": r["unit"].split(" ")[0], "frac": _sig(r["frac"], 3),
                     "traffic": _sig(r["traffic"]) if r["traffic"] else None,
                     "kernel": r["kernel"].split(" ")[0], "kernel_ms": _sig(r["kernel_ms"]),
                     "mfma_frac": _sig(r["mfma"]["frac"], 3),
                     # the dominant kernel's launch ms, min and max over ranks (every rank's in the side file)
                     "rank_ms": [_sig(min(r["per_rank_kernel_ms"])), _sig(max(r["per_rank_kernel_ms"]))]},
        "params_check": {k: v for k, v in (full.get("params_check") or {}).items() if k != "checksum"},
        "detail": os.path.basename(side)[6:-5] if side else side,  # gpurun_out/bench_<detail>.json
    }
    if full.get("fp32_path"):  # the fp32 path's s / update on the same learner (side file: its phases)
        out["fp32_s"] = _sig(full["fp32_path"]["s_per_update"])
    return out


def replica_check(net, dist):
    """After the timed cycle: are the parameters finite, and (N > 1) does every rank hold bitwise the same
    parameters (the gradient all-reduce and identical Adam steps keep the replicas equal)?  An fp64 sum
    and an integer checksum of the flat parameter bits, MIN- and MAX-reduced over ranks."""
    import torch

    finite = torch.isfinite(net.params).all().to(torch.float64).reshape(1)
    if dist is None:
        return {"finite": bool(finite.item()), "identical": None}
    dist.all_reduce(finite, op=dist.ReduceOp.MIN)
    # fp64 value sum, and an int64 checksum of the parameter bits reduced AS int64 (a double would keep only
    # 53 of its bits: a one-ulp difference could vanish); the int64 sum wraps the same way on every rank
    bits = net.params.view(torch.int32).to(torch.int64)
    idx = torch.arange(bits.numel(), device=bits.device, dtype=torch.int64) % 65521 + 1
    vsum = torch.nan_to_num(net.params.double()).sum().reshape(1)
    csum = (bits * idx).sum().reshape(1)
    local = [float(vsum.item()), int(csum.item())]
    same = True
    for t in (vsum, csum):
        lo, hi = t.clone(), t.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        same = same and bool(torch.equal(lo, hi))
    return {"finite": bool(finite.item()), "identical": same, "checksum": local}


def write_side_file(name: str, obj) -> Optional[str]:
    """Per-kernel tables go to a side file (MARLSAT_BENCH_SIDE_DIR, default gpurun_out/) so the one JSON
    line stays short enough for the driver's tail to hold its MAPPO legs."""
    d = os.environ.get("MARLSAT_BENCH_SIDE_DIR", os.path.join(ROOT, "gpurun_out"))
    try:
        os.makedirs(d, exist_ok=True)
        p = os.path.join(d, f"bench_{name}.json")
        with open(p, "w") as f:
            json.dump(obj, f, indent=1)
        return os.path.relpath(p, ROOT)
    except OSError:
        return None


MIXED = ("uf50-218", "uf100-430", "uf200-860")  # BASELINE config 5 size classes (1024 envs per GPU of 8192)


def clock_summary(vals) -> Optional[dict]:
    """Median / p10 / p90 of per-workgroup clocks (MHz) from the env kernel's stamps."""
    import torch

    if vals is None or vals.numel() == 0:
        return None
    q = torch.quantile(vals, torch.tensor([0.1, 0.5, 0.9], dtype=vals.dtype)).tolist()
    return {"median": round(q[1], 1), "p10": round(q[0], 1), "p90": round(q[2], 1), "workgroups": int(vals.numel())}


def stamp_phases(log) -> Optional[dict]:
    """Where an env launch's time goes, from the kernel's stamps (msat_step_out.clock_stamps, 100 MHz real
    time): per launch, the span from the first workgroup's start to the last one's end, and over all
    workgroups the median time from the launch's first start to each workgroup's start (dispatch) and the
    median duration of each phase (wave 0's view), in microseconds; medians over the stamped launches."""
    import statistics

    import torch

    if not log:
        return None
    names = ("assign_loaded", "clause_scan", "tables_staged", "images_built", "obs_stored")
    span, disp, dmax, wg, wg90, wgmax, wgreset, ph = [], [], [], [], [], [], [], {n: [] for n in names}
    for t, done in log:
        ok = t[:, 1] > 0
        t, done = t[ok], done[ok]
        if t.numel() == 0:
            continue
        st, en = t[:, 2], t[:, 7]
        s0 = float(st.min())
        dur = en - st
        span.append((float(en.max()) - s0) / 100.0)
        disp.append(float((st - s0).median()) / 100.0)
        dmax.append(float((st - s0).max()) / 100.0)
        wg.append(float(dur.median()) / 100.0)
        wg90.append(float(torch.quantile(dur, 0.9)) / 100.0)
        wgmax.append(float(dur.max()) / 100.0)
        if bool(done.any()):  # workgroups whose env finished its episode this step (and auto-reset)
            wgreset.append(float(dur[done].median()) / 100.0)
        marks = [t[:, 2]] + [t[:, 3 + i] for i in range(4)] + [t[:, 7]]
        for i, n in enumerate(names):
            a, b = marks[i], marks[i + 1]
            ok = (a > 0) & (b > 0)
            if bool(ok.any()):
                ph[n].append(float((b[ok] - a[ok]).median()) / 100.0)
    med = lambda v: round(statistics.median(v), 3) if v else None
    return {"launch_span_us": med(span), "dispatch_median_us": med(disp), "dispatch_max_us": med(dmax),
            "workgroup_median_us": med(wg), "workgroup_p90_us": med(wg90), "workgroup_max_us": med(wgmax),
            "reset_workgroup_median_us": med(wgreset),
            "phase_median_us": {n: med(v) for n, v in ph.items()}, "launches": len(span)}


def env_leg(args, rank, world, dist, workload: Optional[str] = None, envs: Optional[int] = None,
            preroll_s: Optional[float] = None):
    """Time K fused env steps (+ auto-reset) over the local shard; returns the measurement dict.
    workload / envs override --workload / --envs (the side legs).  Before the W warm-up steps, preroll_s
    seconds of untimed back-to-back launches; after the timed region, --clock-launches launches with the
    kernel's clock stamps on (msat_step_out.clock_stamps), and one stamped launch first of all (cold)."""
    import torch

    from marlsat import SATEnv
    from marlsat.envs.mixed import MixedSATEnv
    from marlsat.random import Key
    from marlsat.utils.generate_cnf_dataset import generate_problem_pool

    workload = workload or args.workload
    envs = envs or args.envs
    mixed = workload == "mixed"
    names = MIXED if mixed else (workload,)
    if mixed:
        total = envs or 1024
        sizes = [total // 3 + (1 if i < total % 3 else 0) for i in range(3)]
    else:
        sizes = [envs or WORKLOADS[workload][3]]
    obs_dtype = torch.int32 if args.obs_dtype == "int32" else torch.int8
    seed = 0x5EED0000 + rank
    classes, pools, pools_np = [], [], []
    for name in names:
        V, C, vpa, _, size_id = WORKLOADS[name]
        pools_np.append(generate_problem_pool(V, C, args.pool, size_id=size_id))
        env = SATEnv(V, C, max_steps=512, vars_per_agent=vpa, obs_dtype=obs_dtype)
        classes.append(env)
        pools.append(env.make_pool(pools_np[-1]))
    gen = torch.Generator(device="cuda").manual_seed(1234 + rank)
    ring = 64
    acts = [torch.randint(0, e.max_vars_per_agent + 1, (ring, b, e.num_agents), generator=gen, device="cuda",
                          dtype=torch.int32) for e, b in zip(classes, sizes)]
    if mixed:
        menv = MixedSATEnv(classes)
        obs, states = menv.reset(pools, sizes, Key(seed, 0))
        outs = menv.alloc_outs(states)
        gstep = menv.stepper(states, obs, outs, autoreset=True, seed=seed)
        step = lambda i, c: gstep([a[i % ring] for a in acts], c)
        glanes = int(os.environ.get("MARLSAT_ENV_GROUP_THREADS", "0")) or (512 if sum(sizes) <= 2048 else 256)
        kernel = f"env_group_kernel<2,{'int' if obs_dtype == torch.int32 else 'signed char'},{glanes}>"
    else:
        o, st = classes[0].reset_from_pool(pools[0], sizes[0], Key(seed, 0))
        obs, states, outs = [o], [st], [classes[0]._step_out(sizes[0])]
        sstep = classes[0].stepper(st, o, outs[0], autoreset=True, seed=seed)
        step = lambda i, c: sstep(acts[0][i % ring], c)
        e0 = classes[0]
        lanes = int(os.environ.get("MARLSAT_ENV_THREADS", "0")) or env_lanes(e0.num_agents, 2 * e0.num_vars + e0.num_clauses, sizes[0])
        kernel = f"env_kernel<2,{'int' if obs_dtype == torch.int32 else 'signed char'},{lanes}>"
    counter = 1
    # the same launches with the kernel's clock stamps on (a second out record carrying the stamp buffers)
    nclk = args.clock_launches
    cbufs = [torch.zeros((b, 8), dtype=torch.int64, device="cuda") for b in sizes]
    couts = [dict(o, clock_stamps=c) for o, c in zip(outs, cbufs)]
    if mixed:
        cg = menv.stepper(states, obs, couts, autoreset=True, seed=seed)
        cstep = lambda i, c: cg([a[i % ring] for a in acts], c)
    else:
        cs1 = classes[0].stepper(states[0], obs[0], couts[0], autoreset=True, seed=seed)
        cstep = lambda i, c: cs1(acts[0][i % ring], c)

    stamp_log = []  # per stamped launch: the (B, 8) stamp rows (msat_step_out.clock_stamps)

    def stamped(n, counter):
        vals = []
        for i in range(n):
            for c in cbufs:
                c.zero_()
            cstep(i, counter + i)
            torch.cuda.synchronize()
            t = torch.cat(cbufs).double()
            stamp_log.append((t.cpu(), torch.cat([o["done"] for o in outs]).cpu().bool()))
            ok = t[:, 1] > 0
            vals.append((t[ok, 0] / t[ok, 1] * 100.0).cpu())  # s_memrealtime ticks at 100 MHz
        return torch.cat(vals) if vals else None

    clk_cold = None
    if nclk:
        clk_cold = clock_summary(stamped(1, counter))  # the process's first env launch
        counter += 1
    # time-based pre-roll (untimed): DVFS settles under sustained load, a 5-launch warm-up is ~0.5 ms
    preroll_s = args.preroll_s if preroll_s is None else preroll_s
    n_pre, t_pre = 0, time.perf_counter()
    while time.perf_counter() - t_pre < preroll_s:
        for _ in range(32):
            step(n_pre, counter)
            counter += 1
            n_pre += 1
        torch.cuda.synchronize()
    preroll = {"s": round(time.perf_counter() - t_pre, 3), "launches": n_pre}
    # steady state: after the pre-roll the episode-step counters are set uniform over [0, MAX_STEPS), so
    # ~B/512 envs time out (and auto-reset: new pool instance + assignment drawn in-kernel) in every launch,
    # as in a long-running rollout (solved envs reset on top of that)
    for st in states:
        st.step.copy_(torch.randint(0, 512, (st.num_envs,), generator=gen, device="cuda", dtype=torch.int32))
        st.invalidate_reset_queue()  # the counters were written directly: the listed timed-out envs are stale
    for i in range(args.warmup):
        step(i, counter)
        counter += 1
    torch.cuda.synchronize()
    step_before = [st.step.clone() for st in states]
    K = args.steps
    # HIP events on the kernel's stream (torch's current stream) bracket the whole timed region:
    # the launches run back to back, so span / K is the mean launch duration.  (An event pair
    # around every launch put a marker between consecutive launches and cost ~15 us per step.)
    per_launch = os.environ.get("MARLSAT_BENCH_PER_LAUNCH_EVENTS") == "1"
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(K if per_launch else 1)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if per_launch:
        for i in range(K):
            ev[i][0].record()
            step(i, counter)
            ev[i][1].record()
            counter += 1
    else:
        ev[0][0].record()
        for i in range(K):
            step(i, counter)
            counter += 1
        ev[0][1].record()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / K  # mean launch duration on the kernel's stream
    rank_ms = [0.0] * world
    rank_ms[rank] = kern_ms
    if dist is not None:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
        rk = torch.tensor(rank_ms, dtype=torch.float64, device="cuda")
        dist.all_reduce(rk)  # every rank fills its own slot: SUM = gather
        rank_ms = [float(v) for v in rk]
    # sanity: the state stays consistent (cheap device checks, after timing)
    for e, st in zip(classes, states):
        assert torch.equal(e.num_clauses - st.clauses_satisfied_status.int().sum(1), st.num_unsatisfied)
    done_frac = float(torch.cat([o["done"].float() for o in outs]).mean())
    # envs that auto-reset inside the timed region (at most once each: K < MAX_STEPS): their counter
    # restarted, so it ends below K; the others advanced by exactly K
    resets = int(sum(int((st.step < K).sum()) for st in states))
    assert all(bool(((st.step < K) | (st.step == sb + K)).all()) for st, sb in zip(states, step_before))
    # the clock the kernel ran at, right after the timed region (stamped launches; not timed)
    stamp_log.clear()  # keep the hot launches only
    clk_hot = clock_summary(stamped(nclk, counter)) if nclk else None
    counter += nclk
    phases = stamp_phases(stamp_log)
    if dist is not None and clk_hot is not None:  # the slowest rank's clock (MIN over ranks)
        t = torch.tensor([clk_hot["median"]], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        clk_hot["median_min_over_ranks"] = float(t[0])
    per_class = []
    launch_bytes = 0
    for name, e, b in zip(names, classes, sizes):
        pe = step_bytes(e.num_vars, e.num_clauses, e.num_agents)
        if obs_dtype == torch.int8:
            pe -= 3 * e.num_agents * (2 * e.num_vars + e.num_clauses)
        launch_bytes += pe * b
        per_class.append({"workload": name, "num_vars": e.num_vars, "num_clauses": e.num_clauses,
                          "num_agents": e.num_agents, "vars_per_agent": WORKLOADS[name][2], "envs_per_gpu": b,
                          "algorithmic_bytes_per_env_step": pe})
    return {"workload": workload, "names": names, "sizes": sizes, "elapsed": elapsed, "kern_ms": kern_ms,
            "rank_ms": rank_ms, "K": K, "sclk": clk_hot, "sclk_cold": clk_cold, "preroll": preroll,
            "stamp_phases": phases,
            "kernel": kernel,
            "launch_bytes": launch_bytes, "per_class": per_class, "done_frac": done_frac, "resets": resets}


def env_side_legs(args, rank, world, dist) -> list:
    """BASELINE configs 2, 3 and 5 beside the headline env leg (``--env-legs``, 'workload:envs_per_gpu,...'):
    the same timed loop, compact records (whole-job env-steps/s, mean launch ms, HBM fraction)."""
    out, stamps = [], {}
    for spec in filter(None, args.env_legs.split(",")):
        wl, envs = spec.split(":")
        r = env_leg(args, rank, world, dist, wl, int(envs), preroll_s=min(args.preroll_s, 0.25))
        B = sum(r["sizes"])
        gbs = r["launch_bytes"] / (r["kern_ms"] * 1e-3) / 1e9
        out.append({"workload": wl, "envs_per_gpu": B, "value": _sig(B * r["K"] * world / r["elapsed"]),
                    "kernel_ms": _sig(r["kern_ms"]), "frac": _sig(gbs / HBM_PEAK_GBS, 3),
                    "sclk_mhz": r["sclk"]["median"] if r["sclk"] else None})
        stamps[f"{wl}:{B}"] = {"kernel_ms": r["kern_ms"], "sclk": r["sclk"], "phases": r["stamp_phases"]}
    if rank == 0 and stamps:
        write_side_file(f"env_stamps_n{world}", stamps)
    return out


def run_cpu_baselines(args) -> dict:
    """The CPU legs, timed before anything touches the GPU (forked workers, torch CPU threads): the env
    step restated (``cpu_baseline``) and the PPO minibatch forward + backward restated on the first MAPPO
    leg's size (``mappo_cpu_baseline``)."""
    from marlsat.utils.generate_cnf_dataset import generate_problem_pool

    progress(0, f"CPU baselines ({args.cpu_budget:g} s budget)")

    names = MIXED if args.workload == "mixed" else (args.workload,)
    rates = []
    host = host_cpu()

    def leg(cores):
        rates = []
        for name in names:
            V, C, vpa, _, size_id = WORKLOADS[name]
            pnp = generate_problem_pool(V, C, min(256, args.pool), size_id=size_id)
            rates.append(cpu_baseline(V, C, vpa, pnp, budget_s=args.cpu_budget / len(names), cores=cores))
        cpu = rates[0]
        if len(rates) > 1:  # time to step one env of each class in the workload's proportions
            tot = args.envs or 1024
            sz = [tot // 3 + (1 if i < tot % 3 else 0) for i in range(3)]
            cpu = dict(rates[0], value=sum(sz) / sum(b / r["value"] for b, r in zip(sz, rates)),
                       sample=" | ".join(r["sample"] for r in rates))
        return cpu

    # one worker per host core the box gives this process (its cgroup CPU quota; the
    # affinity mask shows the whole machine)
    cpu = leg(None)
    if args.cpu_all_cores and host["cores"] < host["affinity_cores"]:
        wide = leg(host["affinity_cores"])
        cpu["all_affinity"] = {"value": wide["value"], "processes": wide["processes"], "cores": wide["cores"],
                               "oversubscribed": wide["oversubscribed"]}
    out = {"env": cpu, "mappo": None}
    legs = [s for s in args.mappo.split(",") if s]
    if legs:
        out["mappo"] = mappo_cpu_baseline(legs[0].split(":")[0], budget_s=min(10.0, args.cpu_budget))
    return out


def launch_ranks(args) -> int:
    """``bench.py --gpus N`` (N > 1) started without torchrun: time the CPU baselines here, then run N
    ranks as a fresh child ``python -m torch.distributed.run`` (one process per GPU, RCCL) and return its
    exit code.  This process never initialises the GPU (no exec from a GPU process; the child is a new
    process tree)."""
    import tempfile

    env = dict(os.environ)
    if args.cpu_budget > 0:
        base = run_cpu_baselines(args)
        fd, path = tempfile.mkstemp(prefix="marlsat_cpu_", suffix=".json")
        with os.fdopen(fd, "w") as f:
            json.dump(base, f)
        env["MARLSAT_BENCH_CPU_JSON"] = path
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    try:
        return subprocess.call(cmd, env=env)
    finally:
        if "MARLSAT_BENCH_CPU_JSON" in env:
            os.unlink(env["MARLSAT_BENCH_CPU_JSON"])


def resolve_world(gpus: Optional[int], environ) -> "int | str | None":
    """The run's world size: torchrun's WORLD_SIZE when set (``--gpus`` may be omitted; an explicit one that
    disagrees -> None, an error), else ``--gpus`` (default 1); "launch" when N > 1 ranks must be started."""
    if "WORLD_SIZE" in environ:
        world = int(environ["WORLD_SIZE"])
        return world if gpus is None or gpus == world else None
    n = gpus or 1
    return "launch" if n > 1 else n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU (default: torchrun's WORLD_SIZE, else 1); N > 1 without torchrun's env "
                         "starts an N-rank torchrun child")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="uf200-860", choices=sorted(WORKLOADS) + ["mixed"],
                    help="'mixed' = BASELINE config 5: uf50/uf100/uf200 classes in one ragged launch")
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU (default: the workload's; mixed: 1024)")
    ap.add_argument("--pool", type=int, default=1024, help="problem instances in the pool")
    ap.add_argument("--obs-dtype", default="int32", choices=["int32", "int8"])
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU baseline per core (0: skip)")
    ap.add_argument("--mappo", default="uf100-430:4096:8,uf200-860:4096:2",
                    help="MAPPO legs 'workload:envs_per_gpu:NUM_STEPS,...' ('' skips); the first is the headline "
                         "'mappo' (BASELINE config 3, the metric's 4096 envs), the others are 'mappo_other_legs' "
                         "(config 4: uf200-860, 25 agents, 4096 envs per GPU)")
    ap.add_argument("--mappo-micro-gb", type=float, default=240.0, help="activation budget per PPO micro-batch")
    ap.add_argument("--mappo-cycles", type=int, default=3,
                    help="timed train cycles per MAPPO leg (after one warm-up cycle); value = 1 / their median "
                         "(min / median / max reported)")
    ap.add_argument("--mappo-fp32-cycles", type=int, default=1,
                    help="cycles of the headline MAPPO leg rerun on the fp32 path (MARLSAT_PRECISION=fp32, the reference's "
                         "operation order) after its timed cycles: 'fp32_s' beside the default (0: skip)")
    ap.add_argument("--preroll-s", type=float, default=1.0,
                    help="seconds of untimed back-to-back env launches before the --warmup steps of the headline env "
                         "leg (the side legs run 0.25 s), so the timed region starts at the clock a long rollout "
                         "runs at; reported in the line")
    ap.add_argument("--clock-launches", type=int, default=8,
                    help="env launches with the kernel's clock stamps on, right after the timed region (0: none): "
                         "sclk_mhz in the line")
    ap.add_argument("--cpu-all-cores", type=int, default=0,
                    help="0: the env CPU baseline runs one single-thread worker per CPU the box gives this process "
                         "(min of affinity, cgroup quota, OMP_NUM_THREADS); 1: one per affinity core as well, "
                         "labelled oversubscribed when that exceeds the quota (side record 'all_affinity')")
    ap.add_argument("--env-legs", default="uf50-218:1024,uf100-430:4096,mixed:1024,mixed:8192",
                    help="env side legs 'workload:envs_per_gpu,...' ('' skips): BASELINE configs 2 and 3 and config 5 "
                         "(1024 envs per GPU = its 8-GPU share of 8192, and all 8192 on one GPU)")
    args = ap.parse_args()

    world = resolve_world(args.gpus, os.environ)
    if world == "launch":
        sys.exit(launch_ranks(args))
    if world is None:
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={os.environ['WORLD_SIZE']} ranks",
              file=sys.stderr)
        sys.exit(2)
    args.gpus = world
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    base = None
    if rank == 0 and args.cpu_budget > 0:
        path = os.environ.get("MARLSAT_BENCH_CPU_JSON")
        if path:  # timed by the launching parent (launch_ranks) before the ranks started
            with open(path) as f:
                base = json.load(f)
        else:  # forked before any GPU initialisation
            base = run_cpu_baselines(args)

    import torch

    # MARLSAT_DIST_BACKEND=gloo + MARLSAT_SHARE_GPU=1: rehearsal of the N>1 path with several ranks on
    # one GPU (RCCL refuses two ranks per device); the driver's runs use RCCL, one GPU per rank.
    share = os.environ.get("MARLSAT_SHARE_GPU") == "1"
    dev_idx = local_rank % torch.cuda.device_count() if share else local_rank
    torch.cuda.set_device(dev_idx)
    dist = None
    backend = None
    collectives = os.environ.get("MARLSAT_COLLECTIVES", "torch")
    if world > 1:
        import torch.distributed as dist

        backend = os.environ.get("MARLSAT_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_idx))
        else:
            dist.init_process_group(backend)
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but the process group has {dist.get_world_size()} ranks")

    progress(rank, f"env legs, {world} rank(s)")
    r = env_leg(args, rank, world, dist)
    side_env = env_side_legs(args, rank, world, dist)
    legs = []
    for i, spec in enumerate(filter(None, args.mappo.split(","))):
        wl, envs, T = spec.split(":")
        legs.append(mappo_bench(args, rank, world, dist, wl, int(envs), int(T),
                                fp32_cycles=args.mappo_fp32_cycles if i == 0 else 0))
    mappo = legs[0] if legs else None

    if rank == 0:
        B, K, elapsed, kern_ms = sum(r["sizes"]), r["K"], r["elapsed"], r["kern_ms"]
        achieved = r["launch_bytes"] / (kern_ms * 1e-3) / 1e9
        wl_key = args.workload if args.workload != "mixed" else "mixed"
        traffic, traffic_src = load_pmc_traffic(f"{wl_key}/B{B}/{args.obs_dtype}", r["kernel"],
                                                default_shape=args.envs is None and args.pool == 1024)
        sids = ",".join(str(WORKLOADS[n][4]) for n in r["names"])
        cfg = {
            "workload": f"{args.workload} SATEnv.step_env + rollout auto-reset (fused "
                        f"{'msat_env_step_grouped, ragged size classes' if args.workload == 'mixed' else 'msat_env_step'})",
            "envs_per_gpu": B, "global_envs": B * world, "max_steps": 512, "obs_dtype": args.obs_dtype,
            "parallelism": f"dp{world} (independent env shards, no data-path collective)",
        }
        if len(r["per_class"]) == 1:
            pc = r["per_class"][0]
            cfg.update({k: pc[k] for k in ("num_vars", "num_clauses", "num_agents", "vars_per_agent")})
            per_env = pc["algorithmic_bytes_per_env_step"]
        else:
            cfg["classes"] = r["per_class"]
            per_env = r["launch_bytes"] / B
        rec = {
            "metric": METRIC,
            "value": B * K * world / elapsed,
            "unit": "env-steps/s",
            "n_gpus": world,
            # ranks whose gradient all-reduce ran over RCCL (torch "nccl" or the C-ABI communicator); 0 for a
            # single rank or a gloo rehearsal
            "rccl_ranks": world if world > 1 and (backend == "nccl" or collectives == "capi") else 0,
            "dist_backend": backend,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.obs_dtype,
            "data": "synthetic (planted-solution random 3-SAT from the reference generator algorithm, "
                    f"seed=1000*size_id+i (size_id {sids}), pool {args.pool}; random valid mode-0 actions; the "
                    "MAPPO pools pass over seeds leaving a variable in no clause, e.g. uf200 3090)",
            "config": cfg,
            "cpu_baseline": base["env"] if base else None,
            "mappo_cpu_baseline": base["mappo"] if base else None,
            "done_fraction_last_step": r["done_frac"],
            "auto_resets_in_timed_region": r["resets"],
            "steady_state": "episode-step counters staggered uniformly over [0, 512) after the pre-roll, before warm-up",
            # the shader clock the env kernel ran at (per-workgroup s_memtime / s_memrealtime deltas of stamped
            # launches right after the timed region; cold = the process's first env launch), and the untimed
            # time-based pre-roll ahead of the --warmup steps
            "sclk_mhz": r["sclk"]["median"] if r["sclk"] else None,
            "sclk": r["sclk"], "sclk_cold": r["sclk_cold"], "preroll": r["preroll"], "stamp_phases": r["stamp_phases"],
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": r["kernel"],
                "kernel_ms": kern_ms,
                "per_rank_kernel_ms": r["rank_ms"],
                "algorithmic_bytes_per_env_step": per_env,
                "algorithmic_bytes_per_launch": r["launch_bytes"],
                "traffic_source": traffic_src,
            },
            # the side legs close the line, so the driver's tail of stdout holds them
            "env_other_legs": side_env,
            "mappo_other_legs": legs[1:],
            "mappo": mappo,
        }
        print(json.dumps(rec), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
