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
