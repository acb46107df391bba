"""An instance that leaves a variable in no clause (the reference generator allows it,
src/utils/generate_cnf_dataset.py:5-40) makes that variable, assigned 0, an all-zero row through every
layer while the biases sit at their zero init: each LayerNorm (learner:27-82, eps 1e-6) multiplies its
gradient by rsqrt(1e-6) = 1000.  The float64 oracle shows the reference's gradient growing ~3 decades per
layer (at L = 16 it passes fp32 range: the first Adam step of such a run is non-finite in the reference
and in this framework alike), and the bench's pool skips such instances (generate_problem_pool's
skip_isolated)."""
import numpy as np
import torch

from marlsat.utils.generate_cnf_dataset import generate_problem_pool, generate_sat_clauses, has_isolated_variable
from oracle import net as onet
from oracle.sat_env import OracleSATEnv


def test_uf200_bench_seed_with_an_unused_variable_is_skipped():
    cl = generate_sat_clauses(200, 860, 3, 3090)  # uf200-860, size_id 3, instance 90
    assert has_isolated_variable(cl, 200)
    assert not np.isin(126, np.abs(cl))
    assert not has_isolated_variable(generate_sat_clauses(200, 860, 3, 3000), 200)
    pool = generate_problem_pool(200, 860, 92, size_id=3, skip_isolated=True)
    assert not any(has_isolated_variable(p, 200) for p in pool)
    assert np.array_equal(pool[89], generate_sat_clauses(200, 860, 3, 3089))
    assert np.array_equal(pool[90], generate_sat_clauses(200, 860, 3, 3091))  # seed 3090 passed over
    assert np.array_equal(generate_problem_pool(200, 860, 91, size_id=3)[90], cl)  # default keeps the seeds


def _grad_max(L, x_isolated):
    V, C = 20, 91
    cl = generate_sat_clauses(V, C, 3, 7)
    cl = np.where(np.abs(cl) == 20, np.sign(cl) * 19, cl)  # variable 20 left in no clause
    assert has_isolated_variable(cl, V)
    ora = OracleSATEnv(V, C, 10, vars_per_agent=10)
    x = (np.arange(V) % 2).astype(np.int32)
    x[19] = x_isolated
    _, st = ora.reset(cl[None], x[None])
    Ap, An = onet.dense_graph(cl[None], V)
    shapes = onet.param_shapes(64, L, ora.num_agents, ora.max_vars_per_agent, 0)
    P = onet.init_params(shapes, seed=3)
    for k in P:  # the flax init of the rest: biases zero, LayerNorm scale 1 / bias 0
        if k.endswith("/bias"):
            P[k] = torch.zeros_like(P[k])
        elif k.endswith("/scale"):
            P[k] = torch.ones_like(P[k])
    P = {k: v.requires_grad_(True) for k, v in P.items()}
    v = onet.critic(P, L, torch.from_numpy(ora.static_var_features(cl[None])).double(),
                    torch.from_numpy(x[None]).double(), torch.from_numpy(ora.clause_features(st)).double(), Ap, An)
    v.sum().backward()
    return max(float(p.grad.abs().max()) for p in P.values() if p.grad is not None)


def test_oracle_gradient_grows_1000x_per_layer_through_a_constant_row():
    g = {L: _grad_max(L, 0) for L in (2, 4)}
    assert g[4] / g[2] > 1e4, g  # two more LayerNorms on the constant row: >= 1e4 (1000^2 x the GRU's z = 0.5 factors)
    assert _grad_max(4, 1) < 1e3  # assigned 1, the row's input is not constant: no amplification
