"""GPU parity: the HIP env kernels (through the C-ABI) vs the NumPy oracle.

Bit-exact on every integer/byte output (obs, clause status, counts, masks,
assignments, steps, dones) and on the fp32 rewards / features.
"""
import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle.rng import reset_draws
from oracle.sat_env import OracleSATEnv
from marlsat.random import Key

pytestmark = pytest.mark.gpu

CONFIGS = [  # name, V, C, vars_per_agent, B, N
    ("uf20", 20, 91, 10, 8, 6),
    ("uf50", 50, 218, 10, 12, 6),
    ("uf100", 100, 430, 10, 12, 6),
    ("uf200", 200, 860, 8, 12, 6),
    ("rem23", 23, 97, 10, 7, 5),  # 3 agents of 8,8,7: padded slots
    ("auto21", 21, 80, None, 5, 4),  # auto grouping 6,5,5,5
    ("one_agent", 12, 40, 12, 3, 3),
]


def _pool(V, C, N, k=3, seed0=0):
    from marlsat.utils.generate_cnf_dataset import generate_sat_clauses

    return np.stack([generate_sat_clauses(V, C, k, seed=seed0 + i) for i in range(N)])


def _mk(V, C, vpa, max_steps=6, **kw):
    from marlsat import SATEnv

    env = SATEnv(V, C, max_steps=max_steps, vars_per_agent=vpa, **kw)
    ora = OracleSATEnv(V, C, max_steps=max_steps, vars_per_agent=vpa,
                       reward_mode=kw.get("reward_mode", 0), action_mode=kw.get("action_mode", 0),
                       r_clause=kw.get("r_clause", 0.02), r_sat=kw.get("r_sat", 1.0), gamma=kw.get("gamma", 0.99))
    return env, ora


def _np(t):
    return t.detach().cpu().numpy()


def _check_state(env, st, ost, ctx=""):
    np.testing.assert_array_equal(_np(st.variable_assignments), ost.variable_assignments, err_msg=ctx)
    np.testing.assert_array_equal(_np(st.clauses_satisfied_status).astype(bool), ost.clauses_satisfied_status,
                                  err_msg=ctx)
    np.testing.assert_array_equal(_np(st.num_unsatisfied), ost.num_unsatisfied, err_msg=ctx)
    np.testing.assert_array_equal(_np(st.step), ost.step, err_msg=ctx)
    np.testing.assert_array_equal(_np(st.done), ost.done, err_msg=ctx)
    np.testing.assert_array_equal(_np(st.clauses), ost.clauses, err_msg=ctx)
    np.testing.assert_array_equal(_np(st.agent_clause_masks), ost.agent_clause_masks, err_msg=ctx)
    np.testing.assert_array_equal(_np(st.agent_neighbor_masks), ost.agent_neighbor_masks, err_msg=ctx)
    np.testing.assert_array_equal(_np(st.literal_to_agent_idx), ost.literal_to_agent_idx, err_msg=ctx)


def _random_actions(rng, env, B):
    A, M = env.num_agents, env.max_vars_per_agent
    if env.action_mode == 0:
        return rng.integers(0, M + 1, size=(B, A)).astype(np.int32)
    return rng.integers(0, 2, size=(B, A, M)).astype(np.int32)


@pytest.mark.parametrize("name,V,C,vpa,B,N", CONFIGS)
def test_reset_matches_oracle(name, V, C, vpa, B, N):
    env, ora = _mk(V, C, vpa)
    pool = _pool(V, C, N)
    rng = np.random.default_rng(1)
    pidx = rng.integers(0, N, B).astype(np.int32)
    x = rng.integers(0, 2, (B, V)).astype(np.uint8)
    obs, st = env.reset_from_pool(env.make_pool(pool), B, problem_idx=pidx, assignments=x)
    oobs, ost = ora.reset(pool[pidx], x.astype(np.int32))
    np.testing.assert_array_equal(_np(obs), oobs)
    _check_state(env, st, ost, name)
    np.testing.assert_array_equal(_np(env.clause_features(st)), ora.clause_features(ost))
    np.testing.assert_array_equal(_np(st.pool.static_var_features()), ora.static_var_features(pool))
    # get_obs recomputes the same observation without touching the state
    np.testing.assert_array_equal(_np(env.get_obs(st).tensor), oobs)
    _check_state(env, st, ost, name + " after get_obs")


@pytest.mark.parametrize("name,V,C,vpa,B,N", CONFIGS)
@pytest.mark.parametrize("autoreset", [False, True])
def test_rollout_matches_oracle(name, V, C, vpa, B, N, autoreset):
    env, ora = _mk(V, C, vpa, max_steps=5)
    pool = _pool(V, C, N)
    rng = np.random.default_rng(2)
    pidx = rng.integers(0, N, B).astype(np.int32)
    x = rng.integers(0, 2, (B, V)).astype(np.uint8)
    dpool = env.make_pool(pool)
    obs, st = env.reset_from_pool(dpool, B, problem_idx=pidx, assignments=x)
    _, ost = ora.reset(pool[pidx], x.astype(np.int32))
    for t in range(12):
        a = _random_actions(rng, env, B)
        if autoreset:
            npidx = rng.integers(0, N, B).astype(np.int32)
            nx = rng.integers(0, 2, (B, V)).astype(np.uint8)
            obs, out = env.step_raw(st, torch.from_numpy(a).cuda(), autoreset=True, problem_idx=npidx,
                                    assignments=nx)
            oobs, ost, r, d, info = ora.step_autoreset(ost, a, pool[npidx], nx.astype(np.int32))
        else:
            obs, out = env.step_raw(st, torch.from_numpy(a).cuda())
            oobs, ost, r, d, info = ora.step(ost, a)
        ctx = f"{name} t={t}"
        np.testing.assert_array_equal(_np(obs), oobs, err_msg=ctx)
        np.testing.assert_array_equal(_np(out["reward"]), r, err_msg=ctx)
        np.testing.assert_array_equal(_np(out["done"]).astype(bool), d, err_msg=ctx)
        np.testing.assert_array_equal(_np(out["solved"]).astype(bool), info["solved"], err_msg=ctx)
        np.testing.assert_array_equal(_np(out["num_unsatisfied"]), info["num_unsatisfied"], err_msg=ctx)
        np.testing.assert_array_equal(_np(out["episode_step"]), info["episode_step"], err_msg=ctx)
        _check_state(env, st, ost, ctx)


def test_step_env_functional_api_and_solve():
    """Drive a uf20 instance into its (reference-checker) solution: reward 1, done, solved."""
    g = np.load(f"{GOLDEN}/clause_truth.npz", allow_pickle=False)
    cl, sol = g["c0_clauses"], g["c0_x"][6]  # index 6 = brute-force satisfying assignment
    assert g["c0_formula_sat"][6] == 1
    env, ora = _mk(20, 91, 10, max_steps=512)
    x0 = sol.copy()
    x0[3] ^= 1  # agent 0 (vars 0-9) must flip local var 3
    obs, st = env.reset(cl[None], assignments=x0[None])
    acts = {"agent_0": torch.tensor([3], device="cuda"), "agent_1": torch.tensor([10], device="cuda")}  # 10 = no-op
    obs2, st2, rewards, dones, infos = env.step_env(None, st, acts)
    assert float(rewards["agent_0"][0]) == 1.0 and bool(dones["__all__"][0]) and bool(infos["solved"][0])
    assert int(st.step[0]) == 0 and int(st2.step[0]) == 1  # functional: input state untouched
    oobs, ost = ora.reset(cl[None], x0[None].astype(np.int32))
    oobs2, _, r, d, _ = ora.step(ost, np.array([[3, 10]]))
    np.testing.assert_array_equal(_np(obs2.tensor), oobs2)
    np.testing.assert_array_equal(_np(obs2["agent_1"]), oobs2[:, 1])
    status, nun = env._calculate_satisfaction_explicit(sol, cl)
    assert int(nun) == 0 and bool(status.all())


@pytest.mark.parametrize("reward_mode", [0, 1])
@pytest.mark.parametrize("action_mode", [0, 1])
def test_modes_match_oracle(reward_mode, action_mode):
    V, C, B, N = 30, 126, 9, 4
    env, ora = _mk(V, C, 7, max_steps=4, reward_mode=reward_mode, action_mode=action_mode, r_clause=0.03,
                   r_sat=5.0, gamma=0.97)
    pool = _pool(V, C, N, seed0=50)
    rng = np.random.default_rng(3)
    pidx = rng.integers(0, N, B).astype(np.int32)
    x = rng.integers(0, 2, (B, V)).astype(np.uint8)
    obs, st = env.reset_from_pool(env.make_pool(pool), B, problem_idx=pidx, assignments=x)
    _, ost = ora.reset(pool[pidx], x.astype(np.int32))
    for t in range(9):
        a = _random_actions(rng, env, B)
        npidx = rng.integers(0, N, B).astype(np.int32)
        nx = rng.integers(0, 2, (B, V)).astype(np.uint8)
        obs, out = env.step_raw(st, torch.from_numpy(a).cuda(), autoreset=True, problem_idx=npidx, assignments=nx)
        oobs, ost, r, d, info = ora.step_autoreset(ost, a, pool[npidx], nx.astype(np.int32))
        np.testing.assert_array_equal(_np(obs), oobs)
        np.testing.assert_array_equal(_np(out["reward"]), r)  # fp32, same op order -> bitwise
        _check_state(env, st, ost, f"t={t}")


def test_quirk_literals_and_narrow_clauses():
    """Literal 0 (null), repeated vars, K=2 and K=1 pools, odd partition with padded agent slots."""
    env, ora = _mk(7, 5, 3, max_steps=3)  # 3 agents: 3,2,2 -> padded slots on agents 1,2
    cl = np.array([[[1, -2, 0], [3, 3, -1], [-4, 2, 7], [0, 0, 0], [-6, 5, 2]]], np.int32)
    cl = np.repeat(cl, 4, 0)
    cl[1, 0] = [5, 0, -7]
    x = np.random.default_rng(4).integers(0, 2, (4, 7)).astype(np.uint8)
    obs, st = env.reset(cl, assignments=x)
    oobs, ost = ora.reset(cl, x.astype(np.int32))
    np.testing.assert_array_equal(_np(obs.tensor), oobs)
    _check_state(env, st, ost, "quirk")
    for K in (1, 2):
        env2, ora2 = _mk(9, 14, 4)
        pool = _pool(9, 14, 3, k=K, seed0=9)
        xx = np.random.default_rng(K).integers(0, 2, (3, 9)).astype(np.uint8)
        o, s = env2.reset(pool, assignments=xx)
        oo, os_ = ora2.reset(pool, xx.astype(np.int32))
        np.testing.assert_array_equal(_np(o.tensor), oo)
        _check_state(env2, s, os_, f"K={K}")


def test_negative_and_out_of_range_actions():
    env, ora = _mk(23, 97, 10)
    pool = _pool(23, 97, 2)
    x = np.zeros((2, 23), np.uint8)
    obs, st = env.reset(pool, assignments=x)
    _, ost = ora.reset(pool, x.astype(np.int32))
    a = np.array([[-1, -9, 7], [9, 100, -3]], np.int32)  # agent 2 has 7 vars (slot 7 padded)
    obs, out = env.step_raw(st, torch.from_numpy(a).cuda())
    oobs, ost, *_ = ora.step(ost, a)
    np.testing.assert_array_equal(_np(obs), oobs)
    _check_state(env, st, ost)


def test_mode1_actions_outside_0_1_are_refused():
    """env:246-250 XORs the raw action integer, so 2 or -1 would leave a non-binary assignment
    (tests/test_oracle.py pins that behaviour on the oracle).  The facade refuses such actions;
    {0, 1} (everything MultiDiscrete([2]*m) samples) match the oracle bit-exact."""
    env, ora = _mk(23, 97, 10, action_mode=1)  # 3 agents of 8, 8, 7 vars: one padded slot
    pool = _pool(23, 97, 2)
    x = np.random.default_rng(8).integers(0, 2, (2, 23)).astype(np.uint8)
    obs, st = env.reset(pool, assignments=x)
    _, ost = ora.reset(pool, x.astype(np.int32))
    A, M = env.num_agents, env.max_vars_per_agent
    for bad in (2, -1):
        a = np.zeros((2, A, M), np.int32)
        a[1, 0, 3] = bad
        with pytest.raises(ValueError, match="must be 0 or 1"):
            env.step_env(None, st, torch.from_numpy(a).cuda())
    a = np.random.default_rng(9).integers(0, 2, (2, A, M)).astype(np.int32)
    obs2, st2, rewards, dones, infos = env.step_env(None, st, torch.from_numpy(a).cuda())
    oobs, ost2, r, d, _ = ora.step(ost, a)
    np.testing.assert_array_equal(_np(obs2.tensor), oobs)
    _check_state(env, st2, ost2, "mode 1 {0,1}")


def test_rng_reset_replays_on_host():
    from marlsat.random import Key

    V, C, B, N = 100, 430, 64, 9
    env, ora = _mk(V, C, 10)
    pool = _pool(V, C, N)
    key = Key(0xDEADBEEF12345, 77)
    obs, st = env.reset_from_pool(env.make_pool(pool), B, key)
    pidx, x = reset_draws(key.seed, key.counter, B, V, N)
    np.testing.assert_array_equal(_np(st.problem_idx), pidx)
    oobs, ost = ora.reset(pool[pidx], x.astype(np.int32))
    np.testing.assert_array_equal(_np(obs), oobs)
    _check_state(env, st, ost)
    # auto-reset with RNG draws: done envs get reset_draws(seed, counter) rows
    env5, ora5 = _mk(V, C, 10, max_steps=1)  # every step times out
    obs, st = env5.reset_from_pool(env5.make_pool(pool), B, problem_idx=pidx, assignments=x)
    a = np.full((B, env5.num_agents), 10, np.int32)
    k2 = Key(99, 5)
    obs, out = env5.step_raw(st, torch.from_numpy(a).cuda(), autoreset=True, key=k2)
    p2, x2 = reset_draws(k2.seed, k2.counter, B, V, N)
    _, ost = ora5.reset(pool[pidx], x.astype(np.int32))
    oobs, ost, *_ = ora5.step_autoreset(ost, a, pool[p2], x2.astype(np.int32))
    np.testing.assert_array_equal(_np(obs), oobs)
    _check_state(env5, st, ost)


def test_int8_obs_equals_int32_obs():
    V, C, B = 50, 218, 33
    pool = _pool(V, C, 4)
    x = np.random.default_rng(5).integers(0, 2, (B, V)).astype(np.uint8)
    pidx = np.arange(B) % 4
    e32, _ = _mk(V, C, 10)
    e8, _ = _mk(V, C, 10, obs_dtype=torch.int8)
    o32, s32 = e32.reset_from_pool(e32.make_pool(pool), B, problem_idx=pidx, assignments=x)
    o8, s8 = e8.reset_from_pool(e8.make_pool(pool), B, problem_idx=pidx, assignments=x)
    assert o8.dtype == torch.int8
    np.testing.assert_array_equal(_np(o8).astype(np.int32), _np(o32))
    a = torch.randint(0, 11, (B, 5), dtype=torch.int32, device="cuda")
    o32, _ = e32.step_raw(s32, a, autoreset=True)
    o8, _ = e8.step_raw(s8, a, autoreset=True)
    np.testing.assert_array_equal(_np(o8).astype(np.int32), _np(o32))


def test_full_size_uf200_x4096_properties_and_sampled_parity():
    """BASELINE config (4): uf200-860, A=25, B=4096, RNG auto-reset — invariants on every env,
    exact oracle replay on a sample of envs."""
    from marlsat.random import Key

    V, C, B, N = 200, 860, 4096, 64
    env, ora = _mk(V, C, 8, max_steps=3)
    pool = _pool(V, C, N, seed0=3000)
    dpool = env.make_pool(pool)
    obs, st = env.reset_from_pool(dpool, B, Key(1, 0))
    gen = torch.Generator(device="cuda").manual_seed(0)
    sample = np.random.default_rng(6).choice(B, 48, replace=False)
    for t in range(5):
        pidx0, x0 = _np(st.problem_idx).copy(), _np(st.variable_assignments).copy()
        step0 = _np(st.step).copy()
        a = torch.randint(0, 9, (B, 25), generator=gen, device="cuda", dtype=torch.int32)
        key = Key(1, t + 1)
        obs, out = env.step_raw(st, a, autoreset=True, key=key)
        sat = st.clauses_satisfied_status.int()
        assert torch.equal(C - sat.sum(1), st.num_unsatisfied)
        assert torch.equal(st.clause_ntrue.gt(0).int(), sat)
        # replay the sampled envs on the oracle
        _, ost = ora.reset(pool[pidx0[sample]], x0[sample].astype(np.int32))
        ost.step = step0[sample]
        p2, x2 = reset_draws(key.seed, key.counter, B, V, N)
        oobs, ost, r, d, info = ora.step_autoreset(ost, _np(a)[sample], pool[p2[sample]],
                                                   x2[sample].astype(np.int32))
        np.testing.assert_array_equal(_np(obs)[sample], oobs)
        np.testing.assert_array_equal(_np(out["done"])[sample].astype(bool), d)
        np.testing.assert_array_equal(_np(st.variable_assignments)[sample], ost.variable_assignments)


@pytest.mark.parametrize("obs_dtype", [torch.int32, torch.int8])
def test_grouped_mixed_batch_equals_per_class(obs_dtype):
    """Ragged batch (config 5 shape: several size classes in ONE launch) == each class stepped
    alone with its class seed, bit for bit: state, obs and step outputs, through RNG resets."""
    from marlsat.envs.mixed import MixedSATEnv, group_seed
    from marlsat.random import Key

    specs = [(20, 91, 10, 37), (50, 218, 10, 64), (23, 97, 10, 19), (200, 860, 8, 8)]  # V, C, vpa, B
    classes, solo, pools = [], [], []
    for i, (V, C, vpa, B) in enumerate(specs):
        env, _ = _mk(V, C, vpa, max_steps=3, obs_dtype=obs_dtype)
        env2, _ = _mk(V, C, vpa, max_steps=3, obs_dtype=obs_dtype)
        classes.append(env)
        solo.append(env2)
        pools.append(_pool(V, C, 5, seed0=100 * i))
    mixed = MixedSATEnv(classes)
    key = Key(0xABCDEF, 3)
    mpools = [c.make_pool(p) for c, p in zip(classes, pools)]
    obs, states = mixed.reset(mpools, [s[3] for s in specs], key)
    ref = []
    for g, (env2, p, s) in enumerate(zip(solo, pools, specs)):
        o, st = env2.reset_from_pool(env2.make_pool(p), s[3], Key(key.seed ^ group_seed(g), key.counter))
        ref.append((o, st))
    outs = mixed.alloc_outs(states)
    step = mixed.stepper(states, obs, outs, autoreset=True, seed=0x5151)
    rng = np.random.default_rng(0)
    for t in range(6):  # max_steps 3: every env auto-resets at least once
        acts = [torch.from_numpy(_random_actions(rng, c, s[3])).cuda() for c, s in zip(classes, specs)]
        step(acts, 10 + t)
        for g, (env2, (o, st)) in enumerate(zip(solo, ref)):
            o2, out2 = env2.step_raw(st, acts[g], autoreset=True, key=Key(0x5151 ^ group_seed(g), 10 + t), obs=o)
            ctx = f"class {g} step {t}"
            assert torch.equal(obs[g], o2), ctx
            for k in ("reward", "done", "solved", "num_unsatisfied", "episode_step"):
                assert torch.equal(outs[g][k], out2[k]), (ctx, k)
            for f in ("variable_assignments", "clauses_satisfied_status", "num_unsatisfied", "step", "done",
                      "problem_idx"):
                assert torch.equal(getattr(states[g], f), getattr(st, f)), (ctx, f)
    assert any(bool(o["done"].any()) for o in outs)


def test_smallest_env_v1_c1():
    """V=1, C=1, one agent: every code path with single-word bit images."""
    env, ora = _mk(1, 1, 1, max_steps=2)
    pool = np.array([[[1, 0, -1]], [[-1, -1, 1]], [[1, 1, 1]]], dtype=np.int32)  # literal 0, x or -x, duplicates
    B = 6
    pidx = np.array([0, 1, 2, 0, 1, 2], np.int32)
    x = np.array([[0], [1], [0], [1], [0], [1]], np.uint8)
    obs, st = env.reset_from_pool(env.make_pool(pool), B, problem_idx=pidx, assignments=x)
    oobs, ost = ora.reset(pool[pidx], x.astype(np.int32))
    np.testing.assert_array_equal(_np(obs), oobs)
    _check_state(env, st, ost)
    for t in range(3):
        a = np.array([[0], [1], [0], [1], [-1], [5]], np.int32)
        npidx = np.array([2, 2, 1, 1, 0, 0], np.int32)
        nx = np.array([[1], [0], [1], [0], [1], [0]], np.uint8)
        obs, out = env.step_raw(st, torch.from_numpy(a).cuda(), autoreset=True, problem_idx=npidx, assignments=nx)
        oobs, ost, r, d, _ = ora.step_autoreset(ost, a, pool[npidx], nx.astype(np.int32))
        np.testing.assert_array_equal(_np(obs), oobs, err_msg=f"t={t}")
        _check_state(env, st, ost, f"t={t}")
        np.testing.assert_array_equal(_np(out["reward"]), r)


def test_grouped_eight_classes_with_empty_ones():
    """MSAT_MAX_GROUPS classes, two of them empty (middle and last): the block -> class map skips them."""
    from marlsat.envs.mixed import MixedSATEnv, group_seed
    from marlsat.random import Key

    specs = [(20, 91, 10, 5), (12, 40, 4, 0), (23, 97, 10, 9), (30, 120, 7, 3), (16, 60, 5, 1), (50, 218, 10, 4),
             (8, 30, 3, 2), (40, 170, 9, 0)]
    classes, solo, pools = [], [], []
    for i, (V, C, vpa, B) in enumerate(specs):
        classes.append(_mk(V, C, vpa, max_steps=2)[0])
        solo.append(_mk(V, C, vpa, max_steps=2)[0])
        pools.append(_pool(V, C, 3, seed0=50 * i))
    mixed = MixedSATEnv(classes)
    key = Key(77, 1)
    obs, states = mixed.reset([c.make_pool(p) for c, p in zip(classes, pools)], [s[3] for s in specs], key)
    outs = mixed.alloc_outs(states)
    step = mixed.stepper(states, obs, outs, autoreset=True, seed=99)
    ref = [e.reset_from_pool(e.make_pool(p), s[3], Key(77 ^ group_seed(g), 1)) for g, (e, p, s)
           in enumerate(zip(solo, pools, specs))]
    rng = np.random.default_rng(1)
    for t in range(3):
        acts = [torch.from_numpy(_random_actions(rng, c, s[3])).cuda() for c, s in zip(classes, specs)]
        step(acts, 5 + t)
        for g, (e, (o, st)) in enumerate(zip(solo, ref)):
            o2, out2 = e.step_raw(st, acts[g], autoreset=True, key=Key(99 ^ group_seed(g), 5 + t), obs=o)
            assert torch.equal(obs[g], o2), (g, t)
            assert torch.equal(states[g].variable_assignments, st.variable_assignments), (g, t)
            assert torch.equal(outs[g]["reward"], out2["reward"]), (g, t)


def _config5(sizes, max_steps, seed0):
    """BASELINE config 5 classes: uf50-218 (5 agents), uf100-430 (10), uf200-860 (25), native sizes."""
    from marlsat.envs.mixed import MixedSATEnv

    specs = [(50, 218, 10), (100, 430, 10), (200, 860, 8)]
    classes, oras, pools = [], [], []
    for i, ((V, C, vpa), B) in enumerate(zip(specs, sizes)):
        env, ora = _mk(V, C, vpa, max_steps=max_steps)
        classes.append(env)
        oras.append(ora)
        pools.append(_pool(V, C, 16, seed0=seed0 + 1000 * i))
    return MixedSATEnv(classes), classes, oras, pools


def test_config5_grouped_matches_oracle_per_class():
    """Config 5 (mixed uf50 / uf100 / uf200 in ONE grouped launch) against the oracle: every class
    replayed at its native size through env:225-398 (the reference cannot mix sizes,
    runner:114-118), RNG resets replayed on the host with the class seed seed ^ group_seed(g)."""
    from marlsat.envs.mixed import group_seed
    from marlsat.random import Key

    sizes = [24, 16, 12]
    mixed, classes, oras, pools = _config5(sizes, 3, 7000)
    key = Key(0x1234, 2)
    obs, states = mixed.reset([c.make_pool(p) for c, p in zip(classes, pools)], sizes, key)
    osts = []
    for g, (ora, p, B) in enumerate(zip(oras, pools, sizes)):
        p0, x0 = reset_draws(key.seed ^ group_seed(g), key.counter, B, ora.num_vars, len(p))
        oobs, ost = ora.reset(p[p0], x0.astype(np.int32))
        np.testing.assert_array_equal(_np(obs[g]), oobs, err_msg=f"class {g} reset")
        _check_state(classes[g], states[g], ost, f"class {g} reset")
        osts.append(ost)
    outs = mixed.alloc_outs(states)
    seed = 0xC0FFEE
    step = mixed.stepper(states, obs, outs, autoreset=True, seed=seed)
    rng = np.random.default_rng(5)
    n_done = [0] * 3
    for t in range(7):  # max_steps 3: every env auto-resets twice
        acts = [_random_actions(rng, c, B) for c, B in zip(classes, sizes)]
        step([torch.from_numpy(a).cuda() for a in acts], 20 + t)
        for g, (ora, p, B) in enumerate(zip(oras, pools, sizes)):
            p2, x2 = reset_draws(seed ^ group_seed(g), 20 + t, B, ora.num_vars, len(p))
            oobs, osts[g], r, d, info = ora.step_autoreset(osts[g], acts[g], p[p2], x2.astype(np.int32))
            ctx = f"class {g} t={t}"
            np.testing.assert_array_equal(_np(obs[g]), oobs, err_msg=ctx)
            np.testing.assert_array_equal(_np(outs[g]["reward"]), r, err_msg=ctx)
            np.testing.assert_array_equal(_np(outs[g]["done"]).astype(bool), d, err_msg=ctx)
            np.testing.assert_array_equal(_np(outs[g]["num_unsatisfied"]), info["num_unsatisfied"], err_msg=ctx)
            np.testing.assert_array_equal(_np(outs[g]["episode_step"]), info["episode_step"], err_msg=ctx)
            _check_state(classes[g], states[g], osts[g], ctx)
            n_done[g] += int(d.sum())
    assert all(n > 0 for n in n_done)  # the auto-reset branch ran in every class


def test_config5_full_size_8192_properties_and_sampled_parity():
    """Config 5 at its full size on one GPU: 2731 uf50 + 2731 uf100 + 2730 uf200 = 8192 envs in one
    grouped launch.  Invariants on every env (num_unsat == C - sum sat, ntrue > 0 <=> sat, obs
    segments consistent with the state) and exact oracle replay of 32 sampled envs per class."""
    from marlsat.envs.mixed import group_seed
    from marlsat.random import Key

    sizes = [2731, 2731, 2730]
    mixed, classes, oras, pools = _config5(sizes, 4, 9000)
    obs, states = mixed.reset([c.make_pool(p) for c, p in zip(classes, pools)], sizes, Key(5, 0))
    outs = mixed.alloc_outs(states)
    seed = 0xBEEF
    step = mixed.stepper(states, obs, outs, autoreset=True, seed=seed)
    gen = torch.Generator(device="cuda").manual_seed(1)
    samples = [np.random.default_rng(g).choice(B, 32, replace=False) for g, B in enumerate(sizes)]
    n_done = [0] * 3
    for t in range(6):
        before = [(_np(s.problem_idx).copy(), _np(s.variable_assignments).copy(), _np(s.step).copy()) for s in states]
        acts = [torch.randint(0, c.max_vars_per_agent + 1, (B, c.num_agents), generator=gen, device="cuda",
                              dtype=torch.int32) for c, B in zip(classes, sizes)]
        step(acts, 100 + t)
        for g, (c, ora, p, B) in enumerate(zip(classes, oras, pools, sizes)):
            st, C, V = states[g], c.num_clauses, c.num_vars
            sat = st.clauses_satisfied_status.int()
            assert torch.equal(C - sat.sum(1), st.num_unsatisfied), (g, t)
            assert torch.equal(st.clause_ntrue.gt(0).int(), sat), (g, t)
            # own-variable segment of every agent's obs holds the assignment (or -1 elsewhere)
            o = obs[g][:, :, :V].long()
            own = torch.from_numpy((ora.agent_vars[:, :, None] == np.arange(V)[None, None]).any(1)).cuda()
            x = st.variable_assignments.long()[:, None, :].expand_as(o)
            assert torch.equal(torch.where(own[None], x, torch.full_like(o, -1)), o), (g, t)
            # clause segment: status where the clause touches the agent, -1 elsewhere
            oc = obs[g][:, :, V:V + C].long()
            assert bool(((oc == -1) | (oc == sat.long()[:, None, :])).all()), (g, t)
            sm = samples[g]
            pidx0, x0, step0 = before[g]
            _, ost = ora.reset(p[pidx0[sm]], x0[sm].astype(np.int32))
            ost.step = step0[sm]
            p2, x2 = reset_draws(seed ^ group_seed(g), 100 + t, B, V, len(p))
            oobs, ost, r, d, info = ora.step_autoreset(ost, _np(acts[g])[sm], p[p2[sm]], x2[sm].astype(np.int32))
            np.testing.assert_array_equal(_np(obs[g])[sm], oobs, err_msg=f"class {g} t={t}")
            np.testing.assert_array_equal(_np(outs[g]["done"])[sm].astype(bool), d)
            np.testing.assert_array_equal(_np(outs[g]["reward"])[sm], r)
            np.testing.assert_array_equal(_np(st.variable_assignments)[sm], ost.variable_assignments)
            n_done[g] += int(outs[g]["done"].sum())
    assert all(n > 0 for n in n_done)


@pytest.mark.parametrize("V,C,vpa,B", [(50, 218, 10, 64), (200, 860, 8, 16)])
def test_clock_stamps_are_inert_and_plausible(V, C, vpa, B):
    """The diagnostic stamps (msat_step_out.clock_stamps, bench.py's clock and phase breakdown) change no
    output: the same auto-reset steps with and without them are bitwise equal; the stamps give a clock in a
    plausible range and phase times in order (start <= each phase end <= end)."""
    env, _ = _mk(V, C, vpa, max_steps=4)
    pool = _pool(V, C, 6)
    rng = np.random.default_rng(5)
    pidx = rng.integers(0, 6, B).astype(np.int32)
    x = rng.integers(0, 2, (B, V)).astype(np.uint8)
    dpool = env.make_pool(pool)
    runs = []
    for stamp in (False, True):
        obs, st = env.reset_from_pool(dpool, B, problem_idx=pidx, assignments=x)
        out = env._step_out(B)
        if stamp:
            out["clock_stamps"] = torch.zeros((B, 8), dtype=torch.int64, device="cuda")
        rec = []
        for t in range(6):
            a = torch.from_numpy(np.random.default_rng(10 + t).integers(0, env.max_vars_per_agent + 1,
                                                                       (B, env.num_agents)).astype(np.int32)).cuda()
            o, _ = env.step_raw(st, a, autoreset=True, key=Key(7, t + 1), out=out)
            rec.append([_np(o).copy()] + [_np(out[k]).copy() for k in ("reward", "done", "num_unsatisfied")])
        runs.append((rec, _np(st.variable_assignments).copy(), out.get("clock_stamps")))
    for a, b in zip(runs[0][0], runs[1][0]):
        for u, v in zip(a, b):
            np.testing.assert_array_equal(u, v)
    np.testing.assert_array_equal(runs[0][1], runs[1][1])
    s = _np(runs[1][2]).astype(np.int64)
    assert (s[:, 1] > 0).all()
    mhz = 100.0 * s[:, 0] / s[:, 1]
    assert (mhz > 300).all() and (mhz < 3000).all(), mhz
    start, end = s[:, 2], s[:, 7]
    for i in range(3, 7):
        assert ((s[:, i] >= start) & (s[:, i] <= end)).all(), i
    assert (np.diff(s[:, 3:7], axis=1) >= 0).all()


def _state_arrays(st):
    return [_np(t).copy() for t in (st.variable_assignments, st.clauses_satisfied_status, st.clause_ntrue,
                                    st.num_unsatisfied, st.step, st.env_done, st.problem_idx)]


@pytest.mark.parametrize("V,C,vpa,B,max_steps,explicit", [
    (50, 218, 10, 1024, 5, False),  # ~205 time out per step: the first cap (12) in reset workgroups, the rest in place
    (50, 218, 10, 1024, 512, False),  # the bench's steady state: counters staggered, ~2 per step
    (20, 91, 10, 64, 3, True),  # caller-given reset instances and assignments (new_problem_idx / new_assign)
    (200, 860, 8, 512, 7, False),  # 512-lane workgroups
    (23, 97, 10, 40, 1, False),  # every step times out, and so does the step after a reset
    (50, 218, 10, 2048, 512, False),  # counters from one reset: the whole batch times out together every 512 steps
])
def test_reset_queue_is_invisible(V, C, vpa, B, max_steps, explicit):
    """The reset queue (msat_env_state.reset_queue: timed-out envs reset in workgroups of their own, listed by the
    previous launch) changes no output: two copies of one batch, one stepped with the queue and one without,
    stay bitwise equal in every state array, obs and step output over a run of RNG auto-resets (solved and timed
    out), with an env-masked reset, a direct counter write (invalidate_reset_queue) and a non-autoreset step in
    between; and the queue's launches do run reset workgroups (listed envs are seen)."""
    env, _ = _mk(V, C, vpa, max_steps=max_steps)
    N = 16
    pool = env.make_pool(_pool(V, C, N, seed0=700))
    rng = np.random.default_rng(B + max_steps)
    pidx = rng.integers(0, N, B).astype(np.int32)
    x = rng.integers(0, 2, (B, V)).astype(np.uint8)
    _, sq = env.reset_from_pool(pool, B, problem_idx=pidx, assignments=x)
    _, sn = env.reset_from_pool(pool, B, problem_idx=pidx, assignments=x)
    sn.reset_queue = None
    if max_steps == 512 and B == 1024:  # a long rollout's counters
        c = torch.from_numpy(rng.integers(0, 512, B).astype(np.int32)).cuda()
        for s in (sq, sn):
            s.step.copy_(c)
        sq.invalidate_reset_queue()
    listed = 0
    if B == 2048:  # all counters one step short of the limit: the mass timeout at the second launch
        for s in (sq, sn):
            s.step.fill_(510)
        sq.invalidate_reset_queue()
    for t in range(14):
        if t == 5:  # reset a third of the envs in place: their queue entries are cleared
            m = rng.random(B) < 0.33
            for s in (sq, sn):
                env.reset_from_pool(pool, B, Key(5, 1000 + t), state=s, reset_mask=m)
        if t == 8:  # counters written directly
            c = torch.from_numpy(rng.integers(0, max_steps, B).astype(np.int32)).cuda()
            for s in (sq, sn):
                s.step.copy_(c)
            sq.invalidate_reset_queue()
        a = torch.from_numpy(rng.integers(0, env.max_vars_per_agent + 1, (B, env.num_agents)).astype(np.int32)).cuda()
        kw = {}
        if explicit:
            kw = dict(problem_idx=rng.integers(0, N, B).astype(np.int32),
                      assignments=rng.integers(0, 2, (B, V)).astype(np.uint8))
        auto = t != 10  # one plain step_env launch: it clears the entries of every env it steps
        if sq.reset_queue is not None and auto:
            q = _np(sq.reset_queue).view(np.uint32)
            par = sq.reset_serial & 1
            tok = 0x80000000 | (sq.reset_serial & 0x7FFFFFFF)
            listed += int((q[par * B: (par + 1) * B] == tok).sum())
        outs = []
        for s in (sq, sn):
            o, out = env.step_raw(s, a, autoreset=auto, key=Key(9, t), **kw)
            outs.append((_np(o), {k: _np(v) for k, v in out.items()}))
        np.testing.assert_array_equal(outs[0][0], outs[1][0], err_msg=f"obs t={t}")
        for k in outs[0][1]:
            np.testing.assert_array_equal(outs[0][1][k], outs[1][1][k], err_msg=f"{k} t={t}")
        for i, (u, v) in enumerate(zip(_state_arrays(sq), _state_arrays(sn))):
            np.testing.assert_array_equal(u, v, err_msg=f"state array {i} t={t}")
    assert listed > 0  # the queue path ran
