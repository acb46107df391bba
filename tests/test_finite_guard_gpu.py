"""GPU: the learner's fail-loud guard (msat_adam_checked + MAPPOLearner.check_finite).

A pool instance with a variable in no clause (the reference generator allows it; tests/test_isolated_variable.py)
makes that variable, assigned 0 at zero-initialised biases, a constant LayerNorm row whose gradient grows ~1000x
per message-passing layer: at the reference depth L = 16 the first Adam step is non-finite, in the reference
(which then trains on NaN parameters, mappo_runner.py:313-317) and here.  Here the cycle raises instead.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cfg(**kw):
    c = dict(NUM_ENVS=16, NUM_STEPS=1, NUM_UPDATES=10, UPDATE_EPOCHS=1, MINIBATCH_SIZE=16, LEARNING_RATE=3e-4,
             GAMMA=0.99, GAE_LAMBDA=0.95, CLIP_EPS=0.2, ENT_COEF=0.01, VF_COEF=0.5, VF_CLIP=0.2, ANNEAL_LR=False,
             GNN_HIDDEN_DIM=128, GNN_NUM_MESSAGE_PASSING_STEPS=16, action_mode=0)
    c.update(kw)
    return c


def _learner(clauses, V, C, vpa, cfg):
    from marlsat import SATEnv
    from marlsat.learners.gnn import GNNActorCritic
    from marlsat.learners.mappo_gnn_sat_learner import MAPPOLearner

    env = SATEnv(V, C, max_steps=64, vars_per_agent=vpa)
    net = GNNActorCritic(cfg["GNN_HIDDEN_DIM"], cfg["GNN_NUM_MESSAGE_PASSING_STEPS"], env.num_agents,
                         env.max_vars_per_agent, 0, V, device="cuda", seed=0)
    return MAPPOLearner(cfg, env, net, env.make_pool(clauses)), net


def test_isolated_variable_at_depth16_raises():
    from marlsat.learners.mappo_gnn_sat_learner import NO_BAD_STEP
    from marlsat.random import PRNGKey
    from marlsat.utils.generate_cnf_dataset import generate_sat_clauses, has_isolated_variable

    V, C = 20, 91
    cl = generate_sat_clauses(V, C, 3, 7)
    cl = np.where(np.abs(cl) == 20, np.sign(cl) * 19, cl)  # variable 20 left in no clause
    assert has_isolated_variable(cl, V)
    learner, net = _learner(cl[None].astype(np.int32), V, C, 10, _cfg())
    rs = learner.init_runner_state(PRNGKey(0))
    # 16 envs draw Bernoulli(0.5) assignments: the isolated variable is 0 in some of them
    assert bool((rs.env_state.variable_assignments[:, 19] == 0).any())
    with pytest.raises(FloatingPointError, match="variable in no clause"):
        learner.train_cycle(rs, 0, torch.Generator().manual_seed(0))
    assert not bool(torch.isfinite(net.params).all())  # the guard reports; it does not hide the step
    assert int(learner.first_bad.item()) == NO_BAD_STEP  # re-armed for a caller that recovers


def test_clean_pool_passes_the_guard():
    from marlsat.learners.mappo_gnn_sat_learner import NO_BAD_STEP
    from marlsat.random import PRNGKey
    from marlsat.utils.generate_cnf_dataset import generate_problem_pool

    pool = generate_problem_pool(20, 91, 4, size_id=0, skip_isolated=True)
    learner, net = _learner(pool, 20, 91, 10, _cfg(GNN_NUM_MESSAGE_PASSING_STEPS=2))
    rs = learner.init_runner_state(PRNGKey(0))
    learner.train_cycle(rs, 0, torch.Generator().manual_seed(0))
    assert int(learner.first_bad.item()) == NO_BAD_STEP
    assert bool(torch.isfinite(net.params).all())
