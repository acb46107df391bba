"""CPU tests: the oracle against the reference's golden vectors + hand-built KATs."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import mappo as om
from oracle.rng import philox4x32_10, reset_draws
from oracle.sat_env import OracleSATEnv, create_agent_groups


def _golden():
    return np.load(os.path.join(GOLDEN, "clause_truth.npz"), allow_pickle=False)


def test_generator_matches_reference_bytes():
    from marlsat.utils.generate_cnf_dataset import generate_sat_cnf

    for r in json.load(open(os.path.join(GOLDEN, "generator.json"))):
        text = generate_sat_cnf(r["V"], r["C"], r["k"], seed=r["seed"])
        assert hashlib.sha256(text.encode()).hexdigest() == r["sha256"], (r["V"], r["C"], r["seed"])
        if "text" in r:
            assert text == r["text"]


@pytest.mark.parametrize("case", range(7))
def test_oracle_clause_truth_vs_reference_checkers(case):
    g = _golden()
    cl, xs = g[f"c{case}_clauses"], g[f"c{case}_x"]
    B = xs.shape[0]
    status, nun = OracleSATEnv.satisfaction(xs.astype(np.int32), np.broadcast_to(cl, (B,) + cl.shape))
    np.testing.assert_array_equal(status.astype(np.uint8), g[f"c{case}_clause_sat"])
    np.testing.assert_array_equal((nun == 0).astype(np.uint8), g[f"c{case}_formula_sat"])
    np.testing.assert_array_equal((nun == 0).astype(np.uint8), g[f"c{case}_verify"])


def test_oracle_quirk_literals_vs_reference_checker():
    # literal 0 is false; a repeated var behaves as one literal (check_sat.py:20-40)
    g = _golden()
    cl, xs = g["quirk_clauses"], g["quirk_x"]
    status, _ = OracleSATEnv.satisfaction(xs.astype(np.int32), np.broadcast_to(cl, (xs.shape[0],) + cl.shape))
    np.testing.assert_array_equal(status.astype(np.uint8), g["quirk_clause_sat"])


def test_agent_groups_partition():
    # env:296-312 explicit grouping and :313-338 auto grouping
    g = create_agent_groups(200, 8)
    assert len(g) == 25 and all(len(v) == 8 for v in g.values())
    g = create_agent_groups(50, 10)
    assert len(g) == 5
    g = create_agent_groups(35, 7)
    assert len(g) == 5
    g = create_agent_groups(23, 10)  # ceil(23/10)=3 agents: 8,8,7
    assert [len(v) for v in g.values()] == [8, 8, 7]
    g = create_agent_groups(200, None)  # factor 4 divides 200 -> 50 agents of 4
    assert len(g) == 50 and all(len(v) == 4 for v in g.values())
    g = create_agent_groups(21, None)  # 4 does not divide 21 -> max(2, int(sqrt(21)))=4 agents
    assert [len(v) for v in g.values()] == [6, 5, 5, 5]


def test_oracle_env_known_answer():
    """Hand-derived 6-var / 4-clause instance, 2 agents (vars 0-2, 3-5)."""
    env = OracleSATEnv(6, 4, max_steps=3, vars_per_agent=3)
    cl = np.array([[[1, -2, 3], [-1, 4, 5], [-4, -5, -6], [2, 6, -3]]], np.int32)
    x = np.array([[1, 0, 0, 0, 0, 0]], np.int32)
    obs, st = env.reset(cl, x)
    # clause truth: c0: 1 true -> sat; c1: -1 false, 4,5 false -> unsat; c2: sat; c3: -3 true -> sat
    np.testing.assert_array_equal(st.clauses_satisfied_status[0], [True, False, True, True])
    assert st.num_unsatisfied[0] == 1
    # agent 0 owns vars 0,1,2 -> related clauses: c0,c1,c3 ; agent 1: c1,c2,c3
    np.testing.assert_array_equal(st.agent_clause_masks[0], [[1, 1, -1, 1], [-1, 1, 1, 1]])
    # neighbours of agent 0: vars of c0,c1,c3 not own -> 3,4,5 ; agent 1: vars 0,1,2
    np.testing.assert_array_equal(st.agent_neighbor_masks[0], [[-1, -1, -1, 1, 1, 1], [1, 1, 1, -1, -1, -1]])
    exp0 = [1, 0, 0, -1, -1, -1] + [1, 0, -1, 1] + [-1, -1, -1, 0, 0, 0]
    exp1 = [-1, -1, -1, 0, 0, 0] + [-1, 0, 1, 1] + [1, 0, 0, -1, -1, -1]
    np.testing.assert_array_equal(obs[0], [exp0, exp1])
    # agent 1 flips var 3 (local idx 0) -> c1 sat, c2 still sat (-5) -> solved
    obs, st2, r, d, info = env.step(st, np.array([[3, 0]]))  # agent 0: action 3 == no-op
    assert st2.variable_assignments[0].tolist() == [1, 0, 0, 1, 0, 0]
    assert info["solved"][0] and d[0] and r[0] == 1.0 and info["episode_step"][0] == 1
    # timeout path: no-ops until max_steps
    obs, s, r, d, info = env.step(st, np.array([[3, 3]]))
    assert not d[0] and r[0] == 0.0
    obs, s, r, d, info = env.step(s, np.array([[3, 3]]))
    obs, s, r, d, info = env.step(s, np.array([[3, 3]]))
    assert d[0] and not info["solved"][0] and info["episode_step"][0] == 3


def test_oracle_flip_decode_edge_cases():
    env = OracleSATEnv(5, 2, max_steps=10, vars_per_agent=3)  # ceil(5/3)=2 agents: [0,1,2], [3,4]; M=3
    x = np.zeros((1, 5), np.int32)
    # agent 1 has 2 vars: action 2 (a padded slot) is a no-op, action 3 (== M) no-op
    assert env.decode_flips(x, np.array([[0, 2]])).tolist() == [[1, 0, 0, 0, 0]]
    assert env.decode_flips(x, np.array([[3, 1]])).tolist() == [[0, 0, 0, 0, 1]]
    # negative index: jnp normalises -1 -> M-1 = 2 (agent 0 var 2; agent 1 padded -> no flip)
    assert env.decode_flips(x, np.array([[-1, -1]])).tolist() == [[0, 0, 1, 0, 0]]


def test_oracle_mode1_integer_xor_semantics():
    """env:246-250: mode 1 XORs the raw action integer into the int32 assignment; env:135-144: a
    literal is true only for x == 1 (positive) or x == 0 (negative).  An action of 2 or -1 therefore
    leaves a value for which both polarities are false (the device facade refuses such actions)."""
    env = OracleSATEnv(4, 2, max_steps=10, vars_per_agent=2, action_mode=1)  # agents [0,1], [2,3]
    x = np.array([[0, 1, 1, 0]], np.int32)
    new = env.decode_flips(x, np.array([[[2, 1], [-1, 0]]]))
    assert new.tolist() == [[2, 0, -2, 0]]
    cl = np.array([[[1, -1, 3], [-3, 2, 4]]], np.int32)
    status, nun = OracleSATEnv.satisfaction(new, cl)
    assert status.tolist() == [[False, False]] and nun.tolist() == [2]


def test_oracle_pbrs_reward():
    env = OracleSATEnv(6, 4, max_steps=5, vars_per_agent=3, reward_mode=1, r_clause=0.25, r_sat=2.0, gamma=0.5)
    cl = np.array([[[1, -2, 3], [-1, 4, 5], [-4, -5, -6], [2, 6, -3]]], np.int32)
    _, st = env.reset(cl, np.array([[1, 0, 0, 0, 0, 0]], np.int32))
    _, _, r, _, _ = env.step(st, np.array([[3, 0]]))
    # u: 1 -> 0 ; r = 0.5*0 - (-1) + 0.25*1 + 2.0
    assert r[0] == np.float32(3.25)


def test_gae_oracle_matches_closed_form():
    T, B = 5, 3
    rng = np.random.default_rng(0)
    r = rng.standard_normal((T, B)).astype(np.float32)
    v = rng.standard_normal((T, B)).astype(np.float32)
    d = rng.integers(0, 2, (T, B)).astype(bool)
    lv = rng.standard_normal(B).astype(np.float32)
    adv, tgt = om.gae(r, v, d, lv, 0.99, 0.95)
    # float64 closed-form recursion
    a = np.zeros(B)
    nv = lv.astype(np.float64)
    for t in range(T - 1, -1, -1):
        nd = 1.0 - d[t]
        a = r[t] + 0.99 * nv * nd - v[t] + 0.99 * 0.95 * nd * a
        np.testing.assert_allclose(adv[t], a, rtol=1e-5, atol=1e-6)
        nv = v[t]
    np.testing.assert_allclose(tgt, adv + v)


def test_philox_known_answers():
    # Random123 philox4x32-10 KATs
    out = philox4x32_10(0, 0, 0, 0, 0, 0)
    assert [int(o) for o in out] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    f = 0xFFFFFFFF
    out = philox4x32_10(f, f, f, f, f, f)
    assert [int(o) for o in out] == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    out = philox4x32_10(0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344, 0xA4093822, 0x299F31D0)
    assert [int(o) for o in out] == [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_reset_draws_statistics():
    pidx, x = reset_draws(seed=123, counter=7, num_envs=4096, num_vars=200, num_problems=10)
    assert pidx.min() >= 0 and pidx.max() < 10
    assert abs(np.bincount(pidx, minlength=10) / 4096 - 0.1).max() < 0.03
    assert abs(x.mean() - 0.5) < 0.01
