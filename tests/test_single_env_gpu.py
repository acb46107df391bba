"""GPU parity of the single-agent SatEnv (src/envs/sat_env.py) and the behavioural-cloning
joint-label generator (src/runners/behavioral_cloning.py:54-100) vs their NumPy restatements
(oracle/single_env.py): bit-exact labels, flip deltas, assignments, dones and f32 rewards."""
import numpy as np
import pytest
import torch

from oracle.sat_env import OracleSATEnv
from oracle.single_env import OracleSatEnv, compute_joint_labels_parallel_greedy as oracle_labels

pytestmark = pytest.mark.gpu


def _pool(V, C, N, seed, quirks=False):
    from marlsat.utils.generate_cnf_dataset import generate_sat_clauses

    p = np.stack([generate_sat_clauses(V, C, 3, seed=seed + i) for i in range(N)])
    if quirks:  # duplicate variables, x and -x in one clause, literal 0 slots
        p[0, 0] = [1, 1, -2]
        p[0, 1] = [3, -3, 4]
        p[1, 2] = [0, 5, -6]
        p[1, 3] = [0, 0, 7]
    return p


@pytest.mark.parametrize("V,C,vpa,tau", [(20, 91, 10, 0.0), (23, 97, 10, 0.0), (50, 218, 10, -1.5),
                                         (12, 40, 5, 0.5), (200, 860, 8, 0.0)])
def test_bc_labels_match_reference_greedy(V, C, vpa, tau):
    from marlsat import SATEnv
    from marlsat.runners.behavioral_cloning import compute_joint_labels

    N, B = 6, 40
    pool_np = _pool(V, C, N, seed=17 * V, quirks=True)
    env = SATEnv(V, C, max_steps=5, vars_per_agent=vpa)
    pool = env.make_pool(pool_np)
    rng = np.random.default_rng(V)
    pidx = rng.integers(0, N, B).astype(np.int32)
    x = rng.integers(0, 2, (B, V)).astype(np.uint8)
    labels, deltas = compute_joint_labels(env, pool, pidx, x, tau, return_deltas=True)
    labels, deltas = labels.cpu().numpy(), deltas.cpu().numpy()
    ora = OracleSATEnv(V, C, 5, vars_per_agent=vpa)
    for b in range(B):
        np.testing.assert_array_equal(labels[b], oracle_labels(ora, pool_np[pidx[b]], x[b].astype(np.int32), tau),
                                      err_msg=f"env {b}")
        _, base = ora.satisfaction(x[b][None].astype(np.int32), pool_np[pidx[b]][None])
        flips = np.repeat(x[b][None].astype(np.int32), V, 0)
        flips[np.arange(V), np.arange(V)] ^= 1
        _, nu = ora.satisfaction(flips, np.repeat(pool_np[pidx[b]][None], V, 0))
        np.testing.assert_array_equal(deltas[b], nu - base[0])


def test_bc_single_env_signature_and_preprocess():
    from marlsat import SATEnv
    from marlsat.runners.behavioral_cloning import compute_joint_labels_parallel_greedy, preprocess
    from marlsat.utils.generate_cnf_dataset import generate_sat_clauses

    V, C = 20, 91
    env = SATEnv(V, C, max_steps=5, vars_per_agent=5)
    ora = OracleSATEnv(V, C, 5, vars_per_agent=5)
    cl = generate_sat_clauses(V, C, seed=4)
    x = np.random.default_rng(1).integers(0, 2, V)
    np.testing.assert_array_equal(compute_joint_labels_parallel_greedy(env, cl, x, 0.0), oracle_labels(ora, cl, x, 0.0))
    expert = [{"problem_clauses": generate_sat_clauses(V, C, seed=s), "expert_solution": np.zeros(V, np.int32)}
              for s in range(3)]
    d = preprocess(expert, env, {"bc_training": {"NUM_SAMPLES_PER_EXPERT": 4, "CORRUPTION_LEVEL": 3}})
    assert d["assignments"].shape == (12, V) and (d["assignments"].sum(1) == 3).all()
    for r in range(12):
        np.testing.assert_array_equal(d["labels"][r], oracle_labels(ora, d["clauses"][d["problem_idx"][r]],
                                                                    d["assignments"][r].astype(np.int32), 0.0))


@pytest.mark.parametrize("V,C,max_steps", [(20, 91, 6), (50, 218, 3)])
def test_single_agent_satenv_matches_reference(V, C, max_steps):
    from marlsat.envs.sat_env import SatEnv

    B, T = 24, 8
    pool_np = _pool(V, C, B, seed=3 * V, quirks=True)
    rng = np.random.default_rng(2)
    x0 = rng.integers(0, 2, (B, V)).astype(np.int32)
    env = SatEnv(V, C, max_clause_len=3, c_bonus=2.5, max_steps=max_steps)
    obs, st = env.reset(None, pool_np, assignments=x0)
    ora = OracleSatEnv(V, C, 3, c_bonus=2.5, max_steps=max_steps)
    ost = ora.reset(pool_np, x0)
    np.testing.assert_array_equal(obs["agent_0"].clause_features.cpu().numpy(), ora.clause_features(ost))
    for t in range(T):
        a = rng.integers(-V - 2, V + 2, B).astype(np.int32)  # includes wrapped and dropped indices
        obs, st, rew, dones, info = env.step_env(None, st, {"agent_0": torch.from_numpy(a)})
        ost, r, d = ora.step(ost, a)
        np.testing.assert_array_equal(st.variable_assignments.cpu().numpy(), ost["x"], err_msg=f"t={t}")
        np.testing.assert_array_equal(rew["agent_0"].cpu().numpy(), r, err_msg=f"t={t}")
        np.testing.assert_array_equal(dones["__all__"].cpu().numpy(), d, err_msg=f"t={t}")
        np.testing.assert_array_equal(obs["agent_0"].clause_features.cpu().numpy(), ora.clause_features(ost))
        np.testing.assert_array_equal(env.unsat_ratio_from_assignment(st).cpu().numpy(), ost["u"])
    assert env.action_space("agent_0").n == V
