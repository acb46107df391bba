"""MAPPO training / evaluation driver -- drop-in for src/runners/mappo_runner.py.

    python -m marlsat.runners.mappo_runner --config configs/MAPPO_CONFIG.yaml [section.KEY=VALUE ...]

Same config file and keys (MAPPO_CONFIG.yaml), same flow (runner:76-464):
  1. seeds; ``load_cnf_problems(CNF_DATA_DIR)``; 80/20 train/eval split with
     ``np.random.RandomState(SEED).shuffle`` (identical index split to the reference);
  2. SATEnv + GNN_ActorCritic + Adam (LR schedule) -- the device implementations;
  3. optional resume (``loading.continue_rl_run_path`` + ``RESET_OPTIMIZER``) or BC
     injection (``loading.inject_bc_model_path``) from flax-format checkpoints;
  4. NUM_UPDATES train cycles, ``training_metrics.txt`` in the reference's CSV format,
     greedy evaluation on EVAL_BATCH_SIZE random eval problems every EVAL_INTERVAL
     updates, ``checkpoints/latest_model_0`` rewritten every update;
  5. final greedy evaluation of every eval problem -> ``test_solutions.txt`` (the
     format ``src/test/verify_solutions.py`` parses) and the solve-rate summary.
Multi-GPU: launch with torchrun; every rank trains its env shard, gradients are
all-reduced (learners/collectives.py); rank 0 logs, evaluates and saves.

``evaluate_policy`` batches all problems of one evaluation into ONE device batch (the
reference jits it per problem and loops on the host, runner:30-73).
"""
from __future__ import annotations

import argparse
import os
import random
import sys
import time
from datetime import datetime
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import yaml

from .. import SATEnv
from ..learners.collectives import init_from_env
from ..learners.gnn import GNNActorCritic
from ..learners.mappo_gnn_sat_learner import MAPPOLearner
from ..random import Key, PRNGKey, split
from ..utils import checkpoints as ck
from ..utils.data_parser import clauses_array, load_cnf_problems, split_train_eval
from ..utils.generate_cnf_dataset import has_isolated_variable

METRICS_HEADER = ("update,mean_return,solve_rate,avg_unsat_clauses,avg_solve_steps,explained_variance,"
                  "value_loss,actor_loss,policy_entropy\n")


# ------------------------------------------------------------ evaluation ----
@torch.no_grad()
def evaluate_policy(key, learner: MAPPOLearner, pool, problem_idx: Sequence[int], max_steps: int,
                    early_exit: bool = True, trace: Optional[list] = None):
    """runner:30-73 for a batch of problems: reset (random assignment), then max_steps greedy
    (argmax) joint actions through step_env; per problem returns
    (was_ever_solved, steps_to_solve (= first solving step + 1, else max_steps),
    solution = the assignment right after that step, zeros if never solved).

    The first solve is final, so stopping once every problem has been solved (checked every
    16 steps) changes no output (early_exit).  ``trace`` (parity tests): a list that receives the
    reset assignment and every step's greedy actions."""
    env, dev = learner.env, learner.device
    k = Key(*key) if isinstance(key, tuple) else key
    k_reset, k_run = split(k, 2)
    idx = torch.as_tensor(np.asarray(problem_idx), dtype=torch.int32, device=dev)
    B = idx.numel()
    obs, st = env.reset_from_pool(pool, B, k_reset, problem_idx=idx)
    out = env._step_out(B)
    solved_any = torch.zeros(B, dtype=torch.bool, device=dev)
    first = torch.full((B,), max_steps, dtype=torch.int32, device=dev)
    sol = torch.zeros((B, env.num_vars), dtype=torch.uint8, device=dev)
    if trace is not None:
        trace.append(st.variable_assignments.clone())
    for t in range(max_steps):
        k_run, k_act = split(k_run, 2)
        act, _, _ = learner.policy(st, k_act, greedy=True, critic=False)
        if trace is not None:
            trace.append(act.clone())
        env.step_raw(st, act, autoreset=False, obs=obs, out=out)
        newly = out["solved"].bool() & ~solved_any
        sol = torch.where(newly[:, None], st.variable_assignments, sol)
        first = torch.where(newly, torch.full_like(first, t + 1), first)
        solved_any |= newly
        if early_exit and (t + 1) % 16 == 0 and bool(solved_any.all()):
            break
    return solved_any.cpu().numpy(), first.cpu().numpy(), sol.cpu().numpy()


def solution_line(name: str, solved: bool, steps: int, solution: np.ndarray) -> str:
    """runner:436-446 line format (parsed by src/test/verify_solutions.py:107)."""
    if solved:
        s = "".join(str(int(v)) for v in solution)
        return f"Problem: {name}, Solved: True, Steps: {int(steps)}, Solution: {s}\n"
    return f"Problem: {name}, Solved: False\n"


def verify_solutions_file(solutions_path: str, cnf_dir: str, env: Optional[SATEnv] = None) -> Dict[str, int]:
    """src/test/verify_solutions.py:84-150 on the device: every ``Solved: True`` line's assignment is
    checked against its CNF with SATEnv._calculate_satisfaction_explicit."""
    import re

    from ..utils.data_parser import parse_cnf

    counts = {"verified": 0, "failed": 0, "skipped": 0}
    pat = re.compile(r"Problem: ([\w.-]+), Solved: True, .* Solution: ([01]+)")
    with open(solutions_path) as f:
        for line in f:
            m = pat.search(line.strip())
            if not m:
                counts["skipped"] += 1
                continue
            name, bits = m.groups()
            V, C, clauses = parse_cnf(os.path.join(cnf_dir, name))
            if len(bits) < V:
                counts["failed"] += 1
                continue
            e = env if (env is not None and env.num_vars == V and env.num_clauses == len(clauses)) else \
                SATEnv(V, len(clauses), max_steps=1, vars_per_agent=V)
            x = np.array([int(c) for c in bits[:V]], dtype=np.uint8)
            _, nun = e._calculate_satisfaction_explicit(x, np.asarray(clauses, dtype=np.int32))
            counts["verified" if int(nun) == 0 else "failed"] += 1
    return counts


# ---------------------------------------------------------------- config ----
def load_config(path: str, overrides: Sequence[str] = ()) -> Dict:
    with open(path) as f:
        cfg = yaml.safe_load(f) or {}
    for ov in overrides:  # hydra-style section.KEY=VALUE
        key, _, val = ov.partition("=")
        d = cfg
        parts = key.split(".")
        for p in parts[:-1]:
            if not isinstance(d.get(p), dict):
                d[p] = {}
            d = d[p]
        d[parts[-1]] = yaml.safe_load(val)
    return cfg


def flat_config(config: Dict) -> Dict:
    """runner:120 -- environment / network / training sections merged."""
    return {**(config.get("environment") or {}), **(config.get("network") or {}), **(config.get("training") or {})}


# ------------------------------------------------------------------ main ----
def run(config: Dict, log=print) -> Dict:
    dist = init_from_env()
    rank = dist.get_rank() if dist is not None else 0
    if torch.cuda.is_available():
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    seed = int(config.get("SEED", 42))
    random.seed(seed)
    np.random.seed(seed)
    key = PRNGKey(seed)
    problems_raw = load_cnf_problems(config.get("CNF_DATA_DIR", "data"))
    if not problems_raw:
        log("no .cnf problems found")
        return {}
    tr_idx, ev_idx = split_train_eval(len(problems_raw), seed)
    train_raw = [problems_raw[i] for i in tr_idx]
    eval_raw = [problems_raw[i] for i in ev_idx]
    log(f"[*] {len(problems_raw)} problems: {len(train_raw)} train (80%), {len(eval_raw)} eval (20%)")
    fc = flat_config(config)
    rewards = fc.get("rewards") or {}
    env = SATEnv(fc["NUM_VARS"], fc["NUM_CLAUSES"], fc["MAX_STEPS"], vars_per_agent=fc.get("VARS_PER_AGENT"),
                 action_mode=fc.get("action_mode", 0), r_clause=rewards.get("R_CLAUSE", 0.02),
                 r_sat=rewards.get("R_SAT", 1.0), gamma=fc.get("GAMMA", 0.99))
    for p in problems_raw:
        if (p["num_vars"], p["num_clauses"]) != (env.num_vars, env.num_clauses):
            raise ValueError(f"{p['name']} is V={p['num_vars']}, C={p['num_clauses']}; the config is "
                             f"V={env.num_vars}, C={env.num_clauses} (one size per run, as the reference)")
    iso = [p["name"] for p in train_raw if has_isolated_variable(clauses_array(p), env.num_vars)]
    if iso:  # the reference trains on them; its first Adam step on one is non-finite (learner check_finite)
        log(f"warning: {len(iso)} training problem(s) leave a variable in no clause ({', '.join(iso[:5])}"
            f"{', ...' if len(iso) > 5 else ''}): at zero-initialised biases such a variable is a constant LayerNorm "
            f"row whose gradient overflows fp32 at depth (tests/test_isolated_variable.py); the learner stops with "
            f"FloatingPointError if an update turns non-finite")
    train_pool = env.make_pool(np.stack([clauses_array(p) for p in train_raw]))
    eval_pool = env.make_pool(np.stack([clauses_array(p) for p in eval_raw])) if eval_raw else None
    net = GNNActorCritic(fc["GNN_HIDDEN_DIM"], fc["GNN_NUM_MESSAGE_PASSING_STEPS"], env.num_agents,
                         env.max_vars_per_agent, env.action_mode, env.num_vars, seed=seed)
    anneal = bool(fc.get("ANNEAL_LR", False))
    loading = config.get("loading") or {}
    if loading.get("continue_rl_run_path"):
        st = ck.restore_checkpoint(os.path.join(loading["continue_rl_run_path"], "checkpoints"), "latest_model_", 0)
        if st is not None:
            ck.load_train_state(net, st, reset_optimizer=bool(loading.get("RESET_OPTIMIZER", False)))
            log("resumed RL checkpoint")
        else:
            log("warning: RL checkpoint not found; training from scratch")
    elif loading.get("inject_bc_model_path"):
        st = ck.restore_checkpoint(loading["inject_bc_model_path"], "bc_model_", None)
        if st is not None:
            ck.inject_bc(net, st)
            log("injected BC encoder + actor parameters")
        else:
            log("warning: BC checkpoint not found; training from scratch")
    learner = MAPPOLearner(fc, env, net, train_pool, dist=dist)
    ne = max(1, len(eval_raw))  # evaluation runs every eval problem as one device batch
    eval_learner = MAPPOLearner(dict(fc, NUM_ENVS=ne, NUM_STEPS=1, MINIBATCH_SIZE=ne), env, net, eval_pool) \
        if eval_pool is not None else None
    time_str = datetime.now().strftime("%Y-%m-%d_%H-%M-%S")
    run_dir = os.path.abspath(os.path.join(config.get("SAVE_DIR", "experiments"), time_str))
    ckpt_dir = os.path.join(run_dir, "checkpoints")
    if rank == 0:
        os.makedirs(ckpt_dir, exist_ok=True)
    key, k_rs = split(key, 2)
    rs = learner.init_runner_state(Key(k_rs.seed + rank, k_rs.counter))
    gen = torch.Generator().manual_seed(seed + rank)
    ev_cfg = config.get("evaluation") or {}
    n_upd = int(fc["NUM_UPDATES"])
    t0 = time.time()
    last = {}
    logf = open(os.path.join(run_dir, "training_metrics.txt"), "w", encoding="utf-8") if rank == 0 else None
    try:
        if logf:
            logf.write(METRICS_HEADER)
        for u in range(n_upd):
            rs, m = learner.train_cycle(rs, u, gen)
            last = m
            if rank != 0:
                continue
            logf.write(f"{u + 1},{m['mean_episodic_return']:.4f},{m['solve_rate']:.4f},"
                       f"{m['avg_unsatisfied_clauses']:.4f},{m['avg_steps_to_solve']:.4f},"
                       f"{m['explained_variance']:.4f},{m['epoch_value_losses'][-1].mean():.4f},"
                       f"{m['epoch_actor_losses'][-1].mean():.4f},{m['epoch_entropies'][-1].mean():.4f}\n")
            logf.flush()
            if eval_learner is not None and (u + 1) % int(ev_cfg.get("EVAL_INTERVAL", 10)) == 0:
                bs = int(ev_cfg.get("EVAL_BATCH_SIZE", 32))
                pick = list(range(len(eval_raw))) if len(eval_raw) < bs else random.sample(range(len(eval_raw)), k=bs)
                key, k_ev = split(key, 2)
                solved, _, _ = evaluate_policy(k_ev, eval_learner, eval_pool, pick, int(fc["MAX_STEPS"]))
                log(f"update {u + 1}: eval solve rate {solved.mean():.2%} ({len(pick)} problems)")
            ck.save_checkpoint(ckpt_dir, ck.train_state_dict(net, anneal), 0, "latest_model_", overwrite=True)
    finally:
        if logf:
            logf.close()
    result = {"run_dir": run_dir, "train_seconds": time.time() - t0, "last_metrics": last}
    if rank == 0 and eval_learner is not None:
        st = ck.restore_checkpoint(ckpt_dir, "latest_model_", 0)
        if st is not None:
            ck.load_train_state(net, st)
        key, k_ev = split(key, 2)
        solved, steps, sols = evaluate_policy(k_ev, eval_learner, eval_pool, range(len(eval_raw)),
                                              int(fc["MAX_STEPS"]))
        with open(os.path.join(run_dir, "test_solutions.txt"), "w", encoding="utf-8") as f:
            for p, s, n, x in zip(eval_raw, solved, steps, sols):
                f.write(solution_line(p["name"], bool(s), int(n), x))
        rate = float(solved.mean()) if len(solved) else 0.0
        avg = float(steps[solved].mean()) if solved.any() else 0.0
        log(f"Final Solve Rate on {len(eval_raw)} eval problems: {rate:.2%}; average steps to solve {avg:.2f}")
        result.update(eval_solve_rate=rate, eval_avg_steps=avg)
    if dist is not None:
        dist.destroy_process_group()
    return result


def main(argv: Optional[List[str]] = None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--config", default="configs/MAPPO_CONFIG.yaml")
    ap.add_argument("overrides", nargs="*", help="section.KEY=VALUE (hydra-style)")
    a = ap.parse_args(argv)
    run(load_config(a.config, a.overrides))


if __name__ == "__main__":
    main(sys.argv[1:])
