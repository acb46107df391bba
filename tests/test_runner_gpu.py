"""GPU: the MAPPO runner end to end on a synthetic DIMACS dataset (load -> 80/20 split -> train
-> periodic + final greedy evaluation -> test_solutions.txt -> verify), the flax-format
checkpoint round trip of the device network + Adam state, and evaluate_policy's early exit."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CFG = os.path.join(os.path.dirname(__file__), "..", "configs", "MAPPO_CONFIG.yaml")


def _overrides(data, save, **kw):
    ov = {"CNF_DATA_DIR": data, "SAVE_DIR": save, "environment.NUM_VARS": 20, "environment.NUM_CLAUSES": 91,
          "environment.VARS_PER_AGENT": 10, "environment.MAX_STEPS": 20, "network.GNN_HIDDEN_DIM": 64,
          "network.GNN_NUM_MESSAGE_PASSING_STEPS": 2, "training.NUM_ENVS": 4, "training.NUM_STEPS": 4,
          "training.NUM_UPDATES": 2, "training.UPDATE_EPOCHS": 1, "training.MINIBATCH_SIZE": 8,
          "evaluation.EVAL_INTERVAL": 1, "evaluation.EVAL_BATCH_SIZE": 1}
    ov.update(kw)
    return [f"{k}={v}" for k, v in ov.items()]


def test_runner_end_to_end(tmp_path):
    from marlsat.runners.mappo_runner import load_config, run, verify_solutions_file
    from marlsat.utils.generate_cnf_dataset import generate_cnf_dataset_sat

    data = tmp_path / "data"
    generate_cnf_dataset_sat(10, 20, 91, str(data), seed=5)
    res = run(load_config(CFG, _overrides(str(data), str(tmp_path / "runs"))), log=lambda *_: None)
    rd = res["run_dir"]
    lines = open(os.path.join(rd, "training_metrics.txt")).read().splitlines()
    assert lines[0].startswith("update,mean_return") and len(lines) == 3
    assert all(np.isfinite([float(v) for v in l.split(",")]).all() for l in lines[1:])
    assert os.path.exists(os.path.join(rd, "checkpoints", "latest_model_0"))
    sol = open(os.path.join(rd, "test_solutions.txt")).read().splitlines()
    assert len(sol) == 2 and all(l.startswith("Problem: uf20-") for l in sol)
    counts = verify_solutions_file(os.path.join(rd, "test_solutions.txt"), str(data))
    assert counts["failed"] == 0 and counts["verified"] + counts["skipped"] == 2
    # resume from the checkpoint (params + optimizer) for one more update
    res2 = run(load_config(CFG, _overrides(str(data), str(tmp_path / "runs2"), **{
        "training.NUM_UPDATES": 1, "loading.continue_rl_run_path": rd, "loading.RESET_OPTIMIZER": False})),
        log=lambda *_: None)
    assert os.path.exists(os.path.join(res2["run_dir"], "checkpoints", "latest_model_0"))


def test_checkpoint_roundtrip_device_net(tmp_path):
    from marlsat.learners.gnn import GNNActorCritic
    from marlsat.utils import checkpoints as ck

    from marlsat.learners import params as P

    a = GNNActorCritic(64, 2, 3, 7, 0, 20, device="cuda", seed=1)
    rng = np.random.default_rng(0)
    for _ in range(2):  # gradients live on flax parameters only (padding / b_hr / b_hz stay zero)
        tree = {k: rng.standard_normal(v.shape).astype(np.float32) for k, v in a.to_flax().items()}
        a.grads.copy_(torch.from_numpy(P.from_flax(tree, 64, 2, 3, 7, 0)))
        a.adam_step(1e-3)
    ck.save_checkpoint(str(tmp_path), ck.train_state_dict(a), 0)
    b = GNNActorCritic(64, 2, 3, 7, 0, 20, device="cuda", seed=2)
    ck.load_train_state(b, ck.restore_checkpoint(str(tmp_path)))
    assert torch.equal(a.params, b.params) and torch.equal(a.adam_m, b.adam_m) and torch.equal(a.adam_v, b.adam_v)
    assert b.adam_count == 2
    c = GNNActorCritic(64, 2, 3, 7, 0, 20, device="cuda", seed=3)
    ck.inject_bc(c, {"params": ck.train_state_dict(a)["params"]})
    fa, fc = a.to_flax(), c.to_flax()
    for k in fa:
        same = np.array_equal(fa[k], fc[k])
        assert same == (not k.startswith("critic")), k  # encoder + actor injected, critic kept
    assert c.adam_count == 0 and float(c.adam_m.abs().sum()) == 0.0


def test_evaluate_policy_early_exit_is_exact():
    from marlsat import SATEnv
    from marlsat.learners.gnn import GNNActorCritic
    from marlsat.learners.mappo_gnn_sat_learner import MAPPOLearner
    from marlsat.random import Key
    from marlsat.runners.mappo_runner import evaluate_policy
    from marlsat.utils.generate_cnf_dataset import generate_problem_pool

    env = SATEnv(20, 91, max_steps=64, vars_per_agent=10)
    pool = env.make_pool(generate_problem_pool(20, 91, 12, size_id=0))
    net = GNNActorCritic(64, 2, env.num_agents, env.max_vars_per_agent, 0, 20, device="cuda", seed=4)
    cfg = dict(NUM_ENVS=12, NUM_STEPS=1, MINIBATCH_SIZE=12)
    lr = MAPPOLearner(cfg, env, net, pool)
    r1 = evaluate_policy(Key(9, 1), lr, pool, range(12), 64, early_exit=True)
    r2 = evaluate_policy(Key(9, 1), lr, pool, range(12), 64, early_exit=False)
    for x, y in zip(r1, r2):
        np.testing.assert_array_equal(x, y)
    solved, steps, sols = r2
    assert ((steps >= 1) & (steps <= 64)).all() and (steps[~solved] == 64).all()
    for i in np.nonzero(solved)[0]:
        _, nun = env._calculate_satisfaction_explicit(sols[i], pool.clauses[i].cpu().numpy())
        assert int(nun) == 0


@pytest.mark.parametrize("mode", [0, 1])
def test_evaluate_policy_replays_on_oracle(mode):
    """runner:30-73 replayed on the oracle: the reset draws (oracle/rng.reset_draws), every step's
    greedy actions (argmax of the float64 oracle logits; a near-tie within 1e-5 of the logit scale
    may go either way in fp32 and is then replayed with the device's choice), the env steps
    (oracle/sat_env.py), the first-solve step and the recorded solution, bit-exact."""
    from marlsat import SATEnv
    from marlsat.learners.gnn import GNNActorCritic
    from marlsat.learners.mappo_gnn_sat_learner import MAPPOLearner
    from marlsat.random import Key, split
    from marlsat.runners.mappo_runner import evaluate_policy
    from marlsat.utils.generate_cnf_dataset import generate_problem_pool
    from oracle import net as onet
    from oracle.rng import reset_draws
    from oracle.sat_env import OracleSATEnv

    V, C, vpa, T = (20, 91, 10, 24) if mode == 0 else (12, 40, 3, 24)
    N = 10
    clauses = generate_problem_pool(V, C, N, size_id=3)
    env = SATEnv(V, C, max_steps=T, vars_per_agent=vpa, action_mode=mode)
    pool = env.make_pool(clauses)
    A, M = env.num_agents, env.max_vars_per_agent
    net = GNNActorCritic(64, 2, A, M, mode, V, device="cuda", seed=6)
    lr = MAPPOLearner(dict(NUM_ENVS=N, NUM_STEPS=1, MINIBATCH_SIZE=N), env, net, pool)
    probs = np.arange(N)[::-1].copy()
    trace = []
    key = Key(21, 4)
    solved, steps, sols = evaluate_policy(key, lr, pool, probs, T, early_exit=False, trace=trace)
    k_reset, _ = split(key, 2)
    _, x0 = reset_draws(k_reset.seed, k_reset.counter, N, V, N)
    np.testing.assert_array_equal(trace[0].cpu().numpy(), x0)
    ora = OracleSATEnv(V, C, T, vars_per_agent=vpa, action_mode=mode)
    _, ost = ora.reset(clauses[probs], x0.astype(np.int32))
    Pf = {k: torch.tensor(v, dtype=torch.float64) for k, v in net.to_flax().items()}
    av, am = torch.from_numpy(ora.agent_vars.astype(np.int64)), torch.from_numpy(ora.action_mask)
    Ap, An = onet.dense_graph(clauses[probs], V)
    svf = torch.from_numpy(ora.static_var_features(clauses[probs])).double()
    o_solved = np.zeros(N, bool)
    o_steps = np.full(N, T)
    o_sol = np.zeros((N, V), np.int32)
    for t in range(T):
        x = torch.from_numpy(ost.variable_assignments.astype(np.float64))
        cf = torch.from_numpy(ora.clause_features(ost)).double()
        with torch.no_grad():
            lg = onet.actor_logits(Pf, 2, svf, x, cf, Ap, An, av, am, mode).numpy()
        dev_act = trace[1 + t].cpu().numpy()
        ref_act = lg.argmax(-1)  # jnp.argmax: first maximum
        top = np.take_along_axis(lg, ref_act[..., None], -1)[..., 0]
        pick = np.take_along_axis(lg, dev_act[..., None].astype(np.int64), -1)[..., 0]
        scale = np.abs(lg[np.isfinite(lg)]).max()
        same = dev_act == ref_act
        assert (same | (top - pick <= 1e-5 * scale)).all(), f"step {t}: greedy action differs beyond a near-tie"
        _, ost, _, _, info = ora.step(ost, dev_act)
        newly = info["solved"] & ~o_solved
        o_sol[newly] = ost.variable_assignments[newly]
        o_steps[newly] = t + 1
        o_solved |= newly
    np.testing.assert_array_equal(solved, o_solved)
    np.testing.assert_array_equal(steps, o_steps)
    np.testing.assert_array_equal(sols, o_sol)
