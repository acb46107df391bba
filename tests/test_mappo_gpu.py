"""GPU: one full MAPPO train cycle on the device vs the oracle replaying the same
transitions / permutation (JAX RNG streams cannot be reproduced, so the device's
own random draws are the shared input).  Checks rollout log-probs and values,
GAE targets / normalised advantages, every minibatch loss, and the parameters
after all Adam steps."""
import os

import numpy as np
import pytest
import torch

from oracle import mappo as om
from oracle import net as onet
from oracle.sat_env import OracleSATEnv

pytestmark = pytest.mark.gpu


def _cfg(**kw):
    c = dict(NUM_ENVS=4, NUM_STEPS=4, NUM_UPDATES=10, UPDATE_EPOCHS=2, MINIBATCH_SIZE=8, LEARNING_RATE=3e-3,
             GAMMA=0.995, GAE_LAMBDA=0.95, CLIP_EPS=0.12, ENT_COEF=0.005, VF_COEF=0.5, VF_CLIP=0.5, ANNEAL_LR=True,
             LR_START_FACTOR=1.0, LR_END_FLOOR=2e-5, GNN_HIDDEN_DIM=64, GNN_NUM_MESSAGE_PASSING_STEPS=2, action_mode=0)
    c.update(kw)
    return c


@pytest.mark.parametrize("mode", [0, 1])
def test_train_cycle_matches_oracle_replay(mode):
    from marlsat import SATEnv
    from marlsat.learners.gnn import GNNActorCritic
    from marlsat.learners.mappo_gnn_sat_learner import MAPPOLearner, learning_rate_at
    from marlsat.random import PRNGKey
    from marlsat.utils.generate_cnf_dataset import generate_problem_pool

    V, C, vpa = (12, 40, 4) if mode == 0 else (12, 40, 3)
    cfg = _cfg(action_mode=mode)
    pool = generate_problem_pool(V, C, 6, size_id=11)
    env = SATEnv(V, C, max_steps=3, vars_per_agent=vpa, action_mode=mode)
    A, M = env.num_agents, env.max_vars_per_agent
    net = GNNActorCritic(64, 2, A, M, mode, V, device="cuda", seed=3)
    p0 = net.to_flax()
    learner = MAPPOLearner(cfg, env, net, env.make_pool(pool), micro_bytes=2e5)  # tiny micro-batches: exercises accumulation
    rs = learner.init_runner_state(PRNGKey(0))
    gen = torch.Generator().manual_seed(123)
    rs, metrics = learner.train_cycle(rs, 0, gen)
    tr = {k: v.cpu().numpy() for k, v in learner.tr.items()}
    T, B = 4, 4
    # ---- oracle replay
    P = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in p0.items()}
    ora = OracleSATEnv(V, C, 3, vars_per_agent=vpa, action_mode=mode)
    av = torch.from_numpy(ora.agent_vars.astype(np.int64))
    am = torch.from_numpy(ora.action_mask)

    def batch_of(pidx, x):
        _, ost = ora.reset(pool[pidx], x.astype(np.int32))
        Ap, An = onet.dense_graph(pool[pidx], V)
        return {"svf": torch.from_numpy(ora.static_var_features(pool[pidx])).double(),
                "x": torch.from_numpy(x.astype(np.float64)), "cf": torch.from_numpy(ora.clause_features(ost)).double(),
                "A_pos": Ap, "A_neg": An}

    flat = lambda a: a.reshape((T * B,) + a.shape[2:])
    bt = batch_of(flat(tr["pidx"]), flat(tr["x"]))
    with torch.no_grad():
        lg = onet.actor_logits(P, 2, bt["svf"], bt["x"], bt["cf"], bt["A_pos"], bt["A_neg"], av, am, mode)
        val = onet.critic(P, 2, bt["svf"], bt["x"], bt["cf"], bt["A_pos"], bt["A_neg"])
        lp = torch.log_softmax(lg, -1).gather(-1, torch.from_numpy(flat(tr["action"])).long()[..., None])[..., 0]
    lp = lp.numpy()
    fin = np.isfinite(lp)
    np.testing.assert_allclose(flat(tr["log_prob"])[fin], lp[fin], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(flat(tr["value"]), val.numpy(), rtol=1e-5, atol=1e-6)
    # GAE from the recorded rewards / dones / values
    last = learner.last_val.cpu().numpy()
    adv, tgt = om.gae(tr["reward"], tr["value"], tr["done"].astype(bool), last, cfg["GAMMA"], cfg["GAE_LAMBDA"])
    np.testing.assert_allclose(learner.targets.cpu().numpy(), tgt, rtol=1e-5, atol=1e-6)
    adv_n, _, _ = om.normalize(adv)
    np.testing.assert_allclose(learner.adv.cpu().numpy(), adv_n, rtol=1e-4, atol=1e-5)
    # PPO epochs with the same permutations (same host generator stream -> same device permutation keys)
    g2 = torch.Generator().manual_seed(123)
    state = {"count": 0, "m": {k: torch.zeros_like(v) for k, v in P.items()},
             "v": {k: torch.zeros_like(v) for k, v in P.items()}}
    params = {k: v.detach().clone() for k, v in P.items()}
    full = dict(bt, action=torch.from_numpy(flat(tr["action"])).long(),
                log_prob=torch.from_numpy(flat(tr["log_prob"]).astype(np.float64)),
                value=torch.from_numpy(flat(tr["value"]).astype(np.float64)),
                targets=torch.from_numpy(tgt.reshape(-1).astype(np.float64)),
                gae=torch.from_numpy(adv_n.reshape(-1).astype(np.float64)))
    losses = []
    gmax = {k: torch.zeros_like(v) for k, v in P.items()}  # per-element max |grad| over the Adam steps
    lr_sum = 0.0
    for e in range(cfg["UPDATE_EPOCHS"]):
        perm = learner.permutation(g2).cpu().numpy()  # the learner's device permutation, same key stream
        for k in range((T * B) // cfg["MINIBATCH_SIZE"]):
            idx = perm[k * 8:(k + 1) * 8]
            mb = {kk: vv[idx] for kk, vv in full.items()}
            Pk = {kk: vv.clone().requires_grad_(True) for kk, vv in params.items()}
            total, (vl, la, ent), _, _ = onet.ppo_loss(Pk, 2, mb, cfg, av, am, mode)
            total.backward()
            losses.append((float(vl.detach()), float(la.detach()), float(ent.detach())))
            grads = {kk: (vv.grad if vv.grad is not None else torch.zeros_like(vv)) for kk, vv in Pk.items()}
            for kk in gmax:
                gmax[kk] = torch.maximum(gmax[kk], grads[kk].abs())
            lr = learning_rate_at(state["count"], cfg)
            lr_sum += lr
            params, state = onet.adam_update(params, grads, state, lr)
    got = np.stack([metrics["epoch_value_losses"].reshape(-1), metrics["epoch_actor_losses"].reshape(-1),
                    metrics["epoch_entropies"].reshape(-1)], 1)
    lerr = np.abs(got - np.array(losses)) / (np.abs(np.array(losses)) + 1e-5)
    print(f"replay mode {mode}: loss error / (|loss| + 1e-5) max {lerr.max():.3g}")
    # measured on MI355X (profiles/r04i_parity.log): loss error <= 2.0e-5 relative, update norm <= 2.5e-4
    np.testing.assert_allclose(got, np.array(losses), rtol=5e-5, atol=1e-5)
    # Adam divides by sqrt(v), so an element whose gradient is near fp32 noise at some step moves by a
    # noise-signed ~lr: single elements are ill-conditioned, the tensor-level update is not.  The loss
    # trajectory above already pins every intermediate parameter set; here each tensor's total update
    # must match the oracle's to 0.1 % in norm and no element may move beyond the Adam step budget.
    final = net.to_flax()
    ratios = []
    for kk, vv in params.items():
        ref, start = vv.numpy(), p0[kk].astype(np.float64)
        upd = np.linalg.norm(ref - start)
        diff = np.linalg.norm(final[kk] - ref)
        ratios.append(diff / max(upd, 1e-30))
        assert diff <= 1e-3 * upd + 1e-7, (kk, diff, upd)
        assert np.abs(final[kk] - ref).max() <= 2.0 * lr_sum + 1e-6, kk
    print(f"replay mode {mode}: |update - oracle update| / |oracle update| worst {max(ratios):.3g}, median "
          f"{float(np.median(ratios)):.3g}")
    # cycle metrics (learner:661-719) from the recorded transitions + the oracle critic on the final params
    done = tr["done"].astype(bool)
    solved = tr["solved"].astype(bool) & done
    n_done, n_solved = done.sum(), solved.sum()
    exp = {"mean_episodic_return": tr["reward"].astype(np.float64).sum(0).mean(),
           "solve_rate": n_solved / max(n_done, 1.0),
           "avg_unsatisfied_clauses": (tr["num_unsatisfied"] * done).sum() / max(n_done, 1.0),
           "avg_steps_to_solve": (tr["episode_step"] * solved).sum() / max(n_solved, 1.0)}
    for k, v in exp.items():
        np.testing.assert_allclose(metrics[k], v, rtol=1e-12, atol=1e-12, err_msg=k)
    Pf = {k: torch.tensor(v, dtype=torch.float64) for k, v in final.items()}
    with torch.no_grad():
        vnew = onet.critic(Pf, 2, bt["svf"], bt["x"], bt["cf"], bt["A_pos"], bt["A_neg"]).numpy()
    tg = learner.targets.cpu().numpy().reshape(-1).astype(np.float64)
    ev = 1.0 - np.var(tg - vnew) / max(np.var(tg), 1e-8)
    np.testing.assert_allclose(metrics["explained_variance"], ev, rtol=1e-4, atol=1e-5)
    assert metrics["current_ent_coef"] == cfg["ENT_COEF"]


def _yard_close(dev, ref, yard, factor, what, rtol=1e-5, extra=None):
    """|dev - ref| <= rtol |ref| + factor * max|yard - ref| (+ extra) (yard: the fp32 CPU oracle's
    value; extra: oracle.net.kink_bound's allowance for ReLU inputs within fp32 noise of 0)."""
    dev, ref, yard = (np.asarray(a, np.float64) for a in (dev, ref, yard))
    fin = np.isfinite(ref)
    assert np.array_equal(fin, np.isfinite(dev)), what
    atol = factor * (np.abs(yard[fin] - ref[fin]).max() if fin.any() else 0.0)
    err = np.abs(dev[fin] - ref[fin])
    bound = rtol * np.abs(ref[fin]) + atol + (0.0 if extra is None else np.asarray(extra, np.float64)[fin])
    worst = float((err / np.maximum(bound, 1e-300)).max()) if err.size else 0.0
    assert (err <= bound).all(), f"{what}: max err {err.max():.3g}, worst ratio {worst:.3g}"
    return worst


# (V, C, vars_per_agent, H, L, mode, (T, B, MB, E))
TRAIN_CYCLE_CASES = [
    (50, 218, 10, 128, 16, 0, (2, 4, 4, 2)),  # uf50-218, 5 agents, the reference's H = 128, L = 16
    (23, 97, 10, 64, 2, 1, (2, 4, 4, 2)),  # mode 1 with a padded variable slot (agents of 8, 8, 7)
    # BASELINE config 4's network: uf200-860, 25 agents of m = 8, two samples, two Adam steps (the fp64
    # oracle runs 25 dense masked 200 x 860 encoders per sample and step; L = 8 keeps it to seconds)
    (200, 860, 8, 128, 8, 0, (1, 2, 1, 1)),
    # the headline MAPPO leg's network (BASELINE config 3): uf100-430, 10 agents of m = 10, H = 128, L = 16,
    # two Adam steps
    (100, 430, 10, 128, 16, 0, (2, 4, 4, 1)),
]


@pytest.fixture
def precision_path(request):
    """Runs the test on one precision path (marlsat.learners.gnn.set_precision: the class switches and the
    library's weight-gradient path) and restores the process's own afterwards."""
    from marlsat.learners import gnn

    prev = gnn.set_precision(request.param)
    yield request.param
    gnn.restore_precision(prev)


@pytest.mark.parametrize("precision_path", ["fp16x2", "bf16x3", "fp32"], indirect=True)
@pytest.mark.parametrize("V,C,vpa,H,L,mode,shape", TRAIN_CYCLE_CASES)
def test_train_cycle_every_adam_step_matches_oracle(V, C, vpa, H, L, mode, shape, precision_path, seed: int = 4):
    """Teacher-forced replay of a whole train cycle: for every Adam step the oracle starts from the
    parameters the device started from (recorded by ``MAPPOLearner.trace``), so each minibatch is
    checked at the north_star bar without the drift of an independent replay (next test):
      * rollout log-probs and values, GAE targets: 1e-5 relative (+ 2x the fp32 oracle's error);
      * the loss triple of EVERY minibatch (the first one included): 1e-5 relative;
      * the gradient of every minibatch: 1e-5 relative + 4x the fp32 oracle's error per tensor (the
        factors of the network depth tests, tests/test_gnn_gpu.py; round 3 allowed 4x / 8x);
      * the Adam step: the device's new parameters vs optax.adam applied in float64 to the device's
        own gradient (1e-5 relative).
    Mode 1 runs with a padded slot: the parameters must stay finite (the slot counts as 0).
    Every case runs on each precision path the README offers (fp16x2 = the default, bf16x3, fp32 = fp32 MFMA
    in the reference's operation order); the margins each path printed are in profiles/r06/."""
    from marlsat import SATEnv
    from marlsat.learners.gnn import GNNActorCritic
    from marlsat.learners.mappo_gnn_sat_learner import MAPPOLearner
    from marlsat.random import PRNGKey
    from marlsat.utils.generate_cnf_dataset import generate_problem_pool

    T, B, MB, E = shape
    cfg = _cfg(NUM_ENVS=B, NUM_STEPS=T, MINIBATCH_SIZE=MB, UPDATE_EPOCHS=E, GNN_HIDDEN_DIM=H,
               GNN_NUM_MESSAGE_PASSING_STEPS=L, action_mode=mode)
    pool = generate_problem_pool(V, C, 5, size_id=12, skip_isolated=True)
    env = SATEnv(V, C, max_steps=2, vars_per_agent=vpa, action_mode=mode)
    A, M = env.num_agents, env.max_vars_per_agent
    assert mode == 0 or V % A  # the mode-1 case must have padded slots
    net = GNNActorCritic(H, L, A, M, mode, V, device="cuda", seed=seed)  # seed: profiles/parity_switch_probe.py
    learner = MAPPOLearner(cfg, env, net, env.make_pool(pool))
    learner.trace = []
    rs = learner.init_runner_state(PRNGKey(seed - 3))
    rs, metrics = learner.train_cycle(rs, 0, torch.Generator().manual_seed(seed + 3))
    assert torch.isfinite(net.params).all()
    tr = {k: v.cpu().numpy() for k, v in learner.tr.items()}
    ora = OracleSATEnv(V, C, 2, vars_per_agent=vpa, action_mode=mode)
    av = torch.from_numpy(ora.agent_vars.astype(np.int64))
    am = torch.from_numpy(ora.action_mask)
    flat = lambda a: a.reshape((T * B,) + a.shape[2:])
    pidx, x = flat(tr["pidx"]), flat(tr["x"])
    _, ost = ora.reset(pool[pidx], x.astype(np.int32))
    Ap, An = onet.dense_graph(pool[pidx], V)
    bt = {"svf": torch.from_numpy(ora.static_var_features(pool[pidx])).double(),
          "x": torch.from_numpy(x.astype(np.float64)), "cf": torch.from_numpy(ora.clause_features(ost)).double(),
          "A_pos": Ap, "A_neg": An}
    args = (bt["svf"], bt["x"], bt["cf"], bt["A_pos"], bt["A_neg"])
    to_t = lambda tree, dt: {k: torch.tensor(v, dtype=dt) for k, v in tree.items()}
    layout = lambda flat_params: _unflat(net, flat_params)
    act = torch.from_numpy(flat(tr["action"])).long()

    def rollout_terms(P):
        with torch.no_grad():
            lg = onet.actor_logits(P, L, *(a.to(next(iter(P.values())).dtype) for a in args), av, am, mode)
            val = onet.critic(P, L, *(a.to(next(iter(P.values())).dtype) for a in args))
            lp = torch.log_softmax(lg, -1).gather(-1, act[..., None])[..., 0]
        if mode == 1:
            lp = torch.where(am[None].expand_as(lp), lp, torch.zeros_like(lp))
        return lp.double().numpy(), val.double().numpy()

    p_start = layout(learner.trace[0]["params"])
    lp64, v64 = rollout_terms(to_t(p_start, torch.float64))
    lp32, v32 = rollout_terms(to_t(p_start, torch.float32))
    vdev = flat(tr["value"]).astype(np.float64)
    print(f"rollout V{V} C{C} A{A} H{H} L{L} mode{mode}: per-sample value |dev - f64| "
          f"{np.array2string(np.abs(vdev - v64), precision=2)}, |f32 - f64| "
          f"{np.array2string(np.abs(v32 - v64), precision=2)}, |value| {np.array2string(np.abs(v64), precision=3)}")
    rl = _yard_close(flat(tr["log_prob"]), lp64, lp32, 2.0, "rollout log_prob")
    rv = _yard_close(vdev, v64, v32, 2.0, "rollout value")
    print(f"margins {precision_path} V{V} C{C} A{A} H{H} L{L} mode{mode} rollout: log_prob worst ratio {rl:.3g}, value worst ratio {rv:.3g}")
    adv, tgt = om.gae(tr["reward"], tr["value"], tr["done"].astype(bool), learner.last_val.cpu().numpy(),
                      cfg["GAMMA"], cfg["GAE_LAMBDA"])
    np.testing.assert_allclose(learner.targets.cpu().numpy(), tgt, rtol=1e-5, atol=1e-7)
    adv_n, _, _ = om.normalize(adv)
    full = dict(bt, action=act, log_prob=torch.from_numpy(flat(tr["log_prob"]).astype(np.float64)),
                value=torch.from_numpy(flat(tr["value"]).astype(np.float64)),
                targets=torch.from_numpy(learner.targets.cpu().numpy().reshape(-1).astype(np.float64)),
                gae=torch.from_numpy(learner.adv.cpu().numpy().reshape(-1).astype(np.float64)))
    np.testing.assert_allclose(full["gae"].numpy(), adv_n.reshape(-1), rtol=1e-5, atol=1e-6)
    dev_losses = np.stack([metrics["epoch_value_losses"].reshape(-1), metrics["epoch_actor_losses"].reshape(-1),
                           metrics["epoch_entropies"].reshape(-1)], 1)
    assert len(learner.trace) == E * (T * B // MB) == dev_losses.shape[0]
    m_st = {"count": 0, "m": None, "v": None}
    dump = os.environ.get("MARLSAT_PARITY_DUMP")  # diagnostics (profiles/parity_orderings.py): the inputs
    if dump:  # of every step's oracle check, saved before the checks run
        os.makedirs(dump, exist_ok=True)
        np.savez(os.path.join(dump, f"{precision_path}_V{V}_L{L}_s{seed}.npz"),
                 **{f"full_{k}": v.numpy() for k, v in full.items()}, av=av.numpy(), am=am.numpy(),
                 **{f"idx_{s}": r["idx"].numpy() for s, r in enumerate(learner.trace)},
                 **{f"params_{s}": r["params"].cpu().numpy() for s, r in enumerate(learner.trace)},
                 **{f"grads_{s}": r["grads"].cpu().numpy() for s, r in enumerate(learner.trace)},
                 pidx=pidx, x_raw=x, shape=np.array([V, C, vpa, H, L, mode, T, B, MB, E]))
    for s, rec in enumerate(learner.trace):
        idx = rec["idx"].numpy()
        mb = {k: v[idx] for k, v in full.items()}
        P_s = layout(rec["params"])
        out = {}
        # fp64 oracle; the fp32 yardstick twice, on the minibatch in its order and reversed (the batch means
        # and the gradients' sums over rows then round differently): E32 per tensor is the larger error of
        # the two, a better sample of fp32's own noise for small tensors (a bias of 11 elements) than one run
        for tag, dt, rows in (("f64", torch.float64, None), ("f32", torch.float32, None),
                              ("f32r", torch.float32, np.arange(len(idx))[::-1].copy())):
            Pk = {k: torch.tensor(v, dtype=dt, requires_grad=True) for k, v in P_s.items()}
            mbk = {k: (v.to(dt) if v.is_floating_point() else v) for k, v in mb.items()}
            if rows is not None:
                mbk = {k: v[torch.from_numpy(rows)] for k, v in mbk.items()}
            onet.RELU_LOG = log = [] if dt == torch.float64 else None
            try:
                total, (vl, la, ent), _, value = onet.ppo_loss(Pk, L, mbk, cfg, av, am, mode)
            finally:
                onet.RELU_LOG = None
            if dt == torch.float64:
                kink, _ = onet.kink_bound(total, Pk, log)
            total.backward()
            out[tag] = ([float(vl.detach()), float(la.detach()), float(ent.detach())],
                        {k: (p.grad.double().numpy() if p.grad is not None else np.zeros(p.shape)) for k, p in Pk.items()},
                        value.detach().double().numpy() if rows is None else value.detach().double().numpy()[rows])
        # losses: 1e-5 relative.  The value loss 0.5 mean (v - target)^2 of a well-fitted critic is a small
        # difference of values, so a value within its own bar (1e-5 |v| + 2 E32, the rollout check above) moves
        # it by |v - target| * dv + dv^2 / 2 per row: that propagated bound is added to the value loss's
        v64, v32 = out["f64"][2], out["f32"][2]
        tol_v = 1e-5 * np.abs(v64) + 2.0 * np.abs(v32 - v64).max()
        tg = mb["targets"].numpy()
        vc = mb["value"].numpy() + np.clip(v64 - mb["value"].numpy(), -cfg["VF_CLIP"], cfg["VF_CLIP"])
        lever = np.maximum(np.abs(v64 - tg), np.abs(vc - tg))
        prop = float(np.mean(lever * tol_v + 0.5 * tol_v ** 2))
        ref_l = np.asarray(out["f64"][0])
        strict = 1e-5 * np.abs(ref_l) + 1e-8
        bound_l = strict + np.array([prop, 0.0, 0.0])
        err_l = np.abs(dev_losses[s] - ref_l)
        assert (err_l <= bound_l).all(), \
            f"Adam step {s}: (value_loss, loss_actor, entropy) {dev_losses[s]} vs {ref_l}, bound {bound_l}"
        # the allowance is fp32's own noise, not the device's: wherever the device's value loss needs it (misses
        # the strict 1e-5 bar), the fp32 CPU oracle's value loss -- the reference's arithmetic class, in either
        # row order -- misses that bar as well
        e32_l = max(abs(out["f32"][0][0] - ref_l[0]), abs(out["f32r"][0][0] - ref_l[0]))
        used = bool(err_l[0] > strict[0])
        if used:
            assert e32_l > strict[0], (f"Adam step {s}: the device value loss needs the propagated allowance "
                                       f"(err {err_l[0]:.3g} > {strict[0]:.3g}) but the fp32 oracle's is within "
                                       f"1e-5 ({e32_l:.3g})")
        g_dev = layout(rec["grads"])
        ratios = {}
        for k in P_s:
            g64, g32, g32r = out["f64"][1][k], out["f32"][1][k], out["f32r"][1][k]
            yard = np.where(np.abs(g32r - g64) > np.abs(g32 - g64), g32r, g32)  # elementwise, then max in _yard_close
            ratios[k] = _yard_close(g_dev[k], g64, yard, 4.0, f"step {s} grad {k}", extra=kink[k])
        top = sorted(ratios.items(), key=lambda kv: -kv[1])[:3]
        gw, gk = top[0][1], top[0][0]
        # the worst tensor's worst element: its error, the strict part of its bar and the fp32 yardstick E32
        g64w = out["f64"][1][gk]
        e32w = max(np.abs(out["f32"][1][gk] - g64w).max(), np.abs(out["f32r"][1][gk] - g64w).max())
        errw = np.abs(np.asarray(g_dev[gk], np.float64) - g64w)
        kw = np.broadcast_to(np.asarray(kink[gk], np.float64), g64w.shape)
        iw = int(np.argmax(errw / (1e-5 * np.abs(g64w) + 4.0 * e32w + kw + 1e-300)))
        print(f"  worst {gk}[{iw}]: err {errw.flat[iw]:.3g}, ref {g64w.flat[iw]:.3g}, 1e-5|ref| "
              f"{1e-5 * abs(g64w.flat[iw]):.3g}, E32 {e32w:.3g} (max |ref| {np.abs(g64w).max():.3g}), "
              f"kink {kw.flat[iw]:.3g}")
        # margins (printed; profiles/r05*_parity_margins.log): each loss's error over its strict 1e-5 bar and
        # over the bar applied; the worst gradient tensor's error over its bar (1.0 = at the bar)
        print(f"margins {precision_path} V{V} C{C} A{A} H{H} L{L} mode{mode} step {s}: loss err/strict "
              f"{np.array2string(err_l / strict, precision=3)} err/bound {np.array2string(err_l / bound_l, precision=3)} "
              f"value allowance used {used} (fp32 oracle value-loss err/strict {e32_l / strict[0]:.3g}); "
              f"grad worst ratio {gw:.3g} ({gk}); next {', '.join(f'{k} {r:.3g}' for k, r in top[1:])}")
        # optax.adam in float64 on the device's own gradient, from the device's own parameters
        gflat = rec["grads"].double().cpu()
        if m_st["m"] is None:
            m_st["m"], m_st["v"] = torch.zeros_like(gflat), torch.zeros_like(gflat)
        pr, m_st2 = onet.adam_update({"p": rec["params"].double().cpu()}, {"p": gflat},
                                     {"count": m_st["count"], "m": {"p": m_st["m"]}, "v": {"p": m_st["v"]}}, rec["lr"])
        m_st = {"count": m_st2["count"], "m": m_st2["m"]["p"], "v": m_st2["v"]["p"]}
        nxt = learner.trace[s + 1]["params"] if s + 1 < len(learner.trace) else net.params
        np.testing.assert_allclose(nxt.double().cpu().numpy(), pr["p"].numpy(), rtol=1e-5, atol=1e-7,
                                   err_msg=f"Adam step {s}")


def _unflat(net, flat_params):
    from marlsat.learners import params as Pm

    return Pm.to_flax(flat_params.detach().cpu().numpy(), net.H, net.L, net.A, net.M, net.mode, net.E)
