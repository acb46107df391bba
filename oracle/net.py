"""torch-CPU restatement of the reference GNN actor-critic + PPO loss — TEST INFRASTRUCTURE.

Follows src/learners/mappo_gnn_sat_learner.py literally, with dense adjacency
and per-agent MASKED full-size encoders exactly as the reference computes them
(:19-82 encoder, :243-255 edge masks, :257-337 actor, :340-350 critic,
:597-645 PPO loss) and the Flax module semantics the reference relies on:
  * nn.Dense: y = x @ kernel + bias, kernel (in, out);
  * nn.GRUCell: r = s(x Wir + bir + h Whr), z = s(x Wiz + biz + h Whz),
                n = tanh(x Win + bin + r * (h Whn + bhn)), h' = (1-z) n + z h;
  * nn.LayerNorm: eps 1e-6, var = E[x^2] - E[x]^2 (use_fast_variance), scale+bias;
    a fresh module per call -> LayerNorm_{3l}, _{3l+1}, _{3l+2} at message step l;
  * distrax.Categorical: log_softmax, entropy = -sum p log p with 0 log 0 = 0.
Gradients come from torch autograd; parameters use the flax tree names
(``encoder/update_c/ir/kernel`` ...).  Runs in float64 or float32.
"""
from __future__ import annotations

import math
from typing import Dict, Tuple

import numpy as np
import torch

GRU_GATES = ("ir", "iz", "in", "hr", "hz", "hn")


def param_shapes(H: int, L: int, A: int, M: int, action_mode: int = 0, embed: int = 16) -> Dict[str, Tuple[int, ...]]:
    """Flax param tree of GNN_ActorCritic (learner:198-241, encoder :44-54, LN per call)."""
    s: Dict[str, Tuple[int, ...]] = {}

    def dense(name, i, o, bias=True):
        s[f"{name}/kernel"] = (i, o)
        if bias:
            s[f"{name}/bias"] = (o,)

    e = "encoder"
    dense(f"{e}/literal_pos_embed", 3, H)
    dense(f"{e}/literal_neg_embed", 3, H)
    dense(f"{e}/clause_embed", 3, H)
    for n in ("phi_c_pos", "phi_c_neg", "phi_v_pos", "phi_v_neg"):
        dense(f"{e}/{n}", H, H)
    for cell, din in (("update_c", 2 * H), ("update_v_pos", H + 4), ("update_v_neg", H + 4)):
        for g in ("ir", "iz", "in"):
            dense(f"{e}/{cell}/{g}", din, H)
        dense(f"{e}/{cell}/hr", H, H, bias=False)
        dense(f"{e}/{cell}/hz", H, H, bias=False)
        dense(f"{e}/{cell}/hn", H, H)
    for k in range(3 * L):
        s[f"{e}/LayerNorm_{k}/scale"] = (H,)
        s[f"{e}/LayerNorm_{k}/bias"] = (H,)
    dense("critic_dense_0", 6 * H, 128)
    dense("critic_dense_1", 128, 64)
    dense("critic_output", 64, 1)
    s["agent_id_embedding/embedding"] = (A, embed)
    ctx = 5 * H + embed
    if action_mode == 0:
        dense("actor_flip_head_dense", 2 * H + ctx, 128)
        dense("actor_flip_head_output", 128, 1)
        dense("actor_noop_head_dense", ctx, 64)
        dense("actor_noop_head_output", 64, 1)
    else:
        dense("actor_dense_0", 2 * H + embed, 128)
        dense("actor_dense_1", 128, 64)
        dense("actor_output", 64, 2)
    return s


def init_params(shapes, seed=0, dtype=torch.float64) -> Dict[str, torch.Tensor]:
    """Flax-like init families (lecun-normal kernels, orthogonal recurrent, zero bias, LN 1/0)."""
    g = torch.Generator().manual_seed(seed)
    out = {}
    for name, shp in shapes.items():
        if name.endswith("/bias"):
            t = torch.randn(shp, generator=g, dtype=torch.float64) * 0.1  # non-zero: exercises bias paths
        elif name.endswith("/scale"):
            t = 1.0 + 0.1 * torch.randn(shp, generator=g, dtype=torch.float64)
        elif name.endswith("/embedding"):
            t = torch.randn(shp, generator=g, dtype=torch.float64) / math.sqrt(shp[1])
        else:
            t = torch.randn(shp, generator=g, dtype=torch.float64) / math.sqrt(shp[0])
        out[name] = t.to(dtype)
    return out


# ReLU kinks.  A pre-activation within fp32 noise of 0 is resolved either way by any fp32
# implementation (the reference's JAX-fp32 run included), and the two sides give gradients that
# differ by g_e * dz_e/dtheta (g_e: the upstream gradient at that ReLU output).  With
# RELU_LOG set to a list, every ReLU call appends (pre-activation, output) with their graphs so
# that kink_bound() can bound that difference for the near-zero elements.
RELU_LOG = None


def _relu(z):
    y = torch.relu(z)
    if RELU_LOG is not None:
        RELU_LOG.append((z, y))
    return y


def kink_bound(obj, params, log, tau=3e-5):
    """Per-parameter bound on the gradient change from resolving near-zero ReLU inputs the other way:
    sum over elements e with |z_e| <= tau * max|z| of |g_e * dz_e/dtheta| (one backward per element).
    obj: the scalar whose gradient is compared (graph retained); log: RELU_LOG of its forward.
    Returns ({name: bound array}, number of ambiguous elements)."""
    names = list(params)
    bound = {k: np.zeros(tuple(params[k].shape)) for k in names}
    ys = [y for _, y in log]
    gys = torch.autograd.grad(obj, ys, retain_graph=True, allow_unused=True)
    n = 0
    for (z, _), gy in zip(log, gys):
        if gy is None:
            continue
        zf, gf = z.reshape(-1), gy.reshape(-1)
        amb = torch.nonzero(zf.detach().abs() <= tau * zf.detach().abs().max()).reshape(-1)
        for e in amb.tolist():
            if float(gf[e]) == 0.0:
                continue
            n += 1
            gr = torch.autograd.grad(zf[e] * gf[e].detach(), [params[k] for k in names], retain_graph=True,
                                     allow_unused=True)
            for k, g in zip(names, gr):
                if g is not None:
                    bound[k] += g.detach().abs().double().numpy()
    return bound, n


def _dense(P, name, x):
    y = x @ P[f"{name}/kernel"]
    b = P.get(f"{name}/bias")
    return y + b if b is not None else y


def _gru(P, name, h, x):
    r = torch.sigmoid(_dense(P, f"{name}/ir", x) + _dense(P, f"{name}/hr", h))
    z = torch.sigmoid(_dense(P, f"{name}/iz", x) + _dense(P, f"{name}/hz", h))
    n = torch.tanh(_dense(P, f"{name}/in", x) + r * _dense(P, f"{name}/hn", h))
    return (1.0 - z) * n + z * h


def _ln(P, k, x, eps=1e-6):
    mean = x.mean(-1, keepdim=True)
    var = torch.clamp((x * x).mean(-1, keepdim=True) - mean * mean, min=0.0)
    y = (x - mean) * torch.rsqrt(var + eps)
    return y * P[f"encoder/LayerNorm_{k}/scale"] + P[f"encoder/LayerNorm_{k}/bias"]


def encoder(P, L, svf, x, cf, A_pos, A_neg, edge_mask=None):
    """learner:27-82.  svf (..,V,3) x (..,V) cf (..,C,3) A (..,V,C) edge_mask (..,V,C)."""
    if edge_mask is not None:
        A_pos, A_neg = A_pos * edge_mask, A_neg * edge_mask
    At_pos, At_neg = A_pos.transpose(-1, -2), A_neg.transpose(-1, -2)
    Hp = _dense(P, "encoder/literal_pos_embed", svf)
    Hn = _dense(P, "encoder/literal_neg_embed", svf)
    Hc = _dense(P, "encoder/clause_embed", cf)
    xin = torch.cat([x[..., None], svf], -1)
    for l in range(L):
        mp = _dense(P, "encoder/phi_c_pos", Hp)
        mn = _dense(P, "encoder/phi_c_neg", Hn)
        Hc = _ln(P, 3 * l, _gru(P, "encoder/update_c", Hc, torch.cat([At_pos @ mp, At_neg @ mn], -1)))
        tp = _dense(P, "encoder/phi_v_pos", Hc)
        tn = _dense(P, "encoder/phi_v_neg", Hc)
        Hp_new = _ln(P, 3 * l + 1, _gru(P, "encoder/update_v_pos", Hp, torch.cat([A_pos @ tp, xin], -1)))
        Hn_new = _ln(P, 3 * l + 2, _gru(P, "encoder/update_v_neg", Hn, torch.cat([A_neg @ tn, xin], -1)))
        Hp, Hn = Hp_new, Hn_new
    return Hp, Hn, Hc


def edge_masks(A_pos, A_neg, agent_vars):
    """learner:243-255 -> (B,A,V,C)."""
    V = A_pos.shape[-2]
    valid = (agent_vars != -1).to(A_pos.dtype)
    oh = torch.nn.functional.one_hot(agent_vars.clamp(min=0).long(), V).to(A_pos.dtype) * valid[..., None]
    var_mask = oh.sum(-2)  # (A,V)
    Aadj = ((A_pos + A_neg) > 0).to(A_pos.dtype)  # (B,V,C)
    clause_mask = ((var_mask[None] @ Aadj) > 0).to(A_pos.dtype)  # (B,A,C)
    related = ((clause_mask @ Aadj.transpose(-1, -2)) > 0).to(A_pos.dtype)  # (B,A,V)
    visible = ((var_mask[None] > 0) | (related > 0)).to(A_pos.dtype)
    return visible[..., :, None] * clause_mask[..., None, :]


def critic(P, L, svf, x, cf, A_pos, A_neg):
    """learner:340-350 -> value (B,)."""
    Hp, Hn, Hc = encoder(P, L, svf, x, cf, A_pos, A_neg)
    Hv = torch.cat([Hp, Hn], -1)
    g = torch.cat([Hv.mean(-2), Hv.amax(-2), Hc.mean(-2), Hc.amax(-2)], -1)
    h = _relu(_dense(P, "critic_dense_0", g))
    h = _relu(_dense(P, "critic_dense_1", h))
    return _dense(P, "critic_output", h)[..., 0]


def actor_logits(P, L, svf, x, cf, A_pos, A_neg, agent_vars, action_mask, action_mode=0):
    """learner:257-337 -> logits (B,A,M+1) mode 0 / (B,A,M,2) mode 1, masked with -inf."""
    B, V, C = A_pos.shape
    Aa, M = agent_vars.shape
    em = edge_masks(A_pos, A_neg, agent_vars)  # (B,A,V,C)
    ex = lambda t: t[:, None].expand(B, Aa, *t.shape[1:])
    Hp, Hn, Hc = encoder(P, L, ex(svf), ex(x), ex(cf), ex(A_pos), ex(A_neg), em)
    Hv = torch.cat([Hp, Hn], -1)  # (B,A,V,2H)
    safe = agent_vars.clamp(min=0).long()
    my = torch.stack([Hv[:, i, safe[i]] for i in range(Aa)], 1)  # (B,A,M,2H)
    vm = (agent_vars != -1).to(Hv.dtype)
    my_sum = (my * vm[None, :, :, None]).sum(2) / vm.sum(-1).clamp(min=1.0)[None, :, None]
    visible = (em.sum(-1) > 0).to(Hv.dtype)  # (B,A,V)
    own = torch.zeros((Aa, V), dtype=Hv.dtype)
    for i in range(Aa):
        for j in range(M):
            if agent_vars[i, j] >= 0:
                own[i, agent_vars[i, j]] += 1.0
    nbr = (visible - own[None]).clamp(0.0, 1.0)
    cm = (em.sum(-2) > 0).to(Hv.dtype)  # (B,A,C)
    pool = lambda X, Mk: (X * Mk[..., None]).sum(-2) / Mk.sum(-1, keepdim=True).clamp(min=1.0)
    ids = P["agent_id_embedding/embedding"][None].expand(B, -1, -1)
    ctx = torch.cat([my_sum, pool(Hv, nbr), pool(Hc, cm), ids], -1)  # (B,A,5H+16)
    if action_mode == 0:
        vin = torch.cat([my, ctx[:, :, None].expand(-1, -1, M, -1)], -1)
        fl = _dense(P, "actor_flip_head_output", _relu(_dense(P, "actor_flip_head_dense", vin)))[..., 0]
        no = _dense(P, "actor_noop_head_output", _relu(_dense(P, "actor_noop_head_dense", ctx)))
        logits = torch.cat([fl, no], -1)
        full = torch.cat([action_mask, torch.ones((Aa, 1), dtype=torch.bool)], -1)
        return torch.where(full[None], logits, torch.tensor(-math.inf, dtype=logits.dtype))
    ain = torch.cat([my, ids[:, :, None].expand(-1, -1, M, -1)], -1)
    h = _relu(_dense(P, "actor_dense_1", _relu(_dense(P, "actor_dense_0", ain))))
    vl = _dense(P, "actor_output", h)
    return torch.where(action_mask[None, :, :, None], vl, torch.tensor(-math.inf, dtype=vl.dtype))


def log_softmax(logits):
    return torch.log_softmax(logits, -1)


def entropy(logits):
    lp = torch.log_softmax(logits, -1)
    p = lp.exp()
    return -torch.where(p > 0, p * lp, torch.zeros_like(p)).sum(-1)


def ppo_loss(P, L, batch, cfg, agent_vars, action_mask, action_mode=0, ent_coef=None):
    """learner:597-645 -> (total, (value_loss, loss_actor, entropy))."""
    svf, x, cf, A_pos, A_neg = batch["svf"], batch["x"], batch["cf"], batch["A_pos"], batch["A_neg"]
    logits = actor_logits(P, L, svf, x, cf, A_pos, A_neg, agent_vars, action_mask, action_mode)
    value = critic(P, L, svf, x, cf, A_pos, A_neg)
    lp_all = log_softmax(logits)
    lp = torch.gather(lp_all, -1, batch["action"].long()[..., None])[..., 0]
    gae = batch["gae"][:, None]
    if action_mode == 0:
        ratio = torch.exp(lp - batch["log_prob"])
    else:
        # padded variable slots (both logits -inf) give NaN log-probs / entropy in distrax, which turns
        # the reference's joint ratio into NaN; the build counts them as 0, so does this
        valid = action_mask[None].expand_as(lp)
        zero = torch.zeros((), dtype=lp.dtype)
        ratio = torch.exp(torch.where(valid, lp, zero).sum(-1) - torch.where(valid, batch["log_prob"], zero).sum(-1))
    eps = cfg["CLIP_EPS"]
    loss_actor = -torch.minimum(ratio * gae, torch.clamp(ratio, 1.0 - eps, 1.0 + eps) * gae).mean()
    ent = entropy(logits).mean()
    c_ent = cfg["ENT_COEF"] if ent_coef is None else ent_coef
    actor_loss = loss_actor - c_ent * ent
    vold = batch["value"]
    vclip = vold + (value - vold).clamp(-cfg["VF_CLIP"], cfg["VF_CLIP"])
    vl = 0.5 * torch.maximum((value - batch["targets"]) ** 2, (vclip - batch["targets"]) ** 2).mean()
    return actor_loss + cfg["VF_COEF"] * vl, (vl, loss_actor, ent), logits, value


def adam_update(params, grads, state, lr, b1=0.9, b2=0.999, eps=1e-8):
    """optax.adam (scale_by_adam + scale by -lr), count incremented before bias correction."""
    cnt = state["count"] + 1
    new_p, m_new, v_new = {}, {}, {}
    for k in params:
        g = grads[k]
        m = b1 * state["m"][k] + (1 - b1) * g
        v = b2 * state["v"][k] + (1 - b2) * g * g
        mh = m / (1 - b1 ** cnt)
        vh = v / (1 - b2 ** cnt)
        new_p[k] = params[k] - lr * mh / (torch.sqrt(vh) + eps)
        m_new[k], v_new[k] = m, v
    return new_p, {"count": cnt, "m": m_new, "v": v_new}


def dense_graph(clauses: np.ndarray, V: int):
    """create_static_graph (graph_constructor.py:93-114) as torch (B,V,C) float64."""
    B, C, K = clauses.shape
    Ap = np.zeros((B, V, C))
    An = np.zeros((B, V, C))
    for b in range(B):
        for c in range(C):
            for l in clauses[b, c]:
                if l > 0:
                    Ap[b, l - 1, c] += 1
                elif l < 0:
                    An[b, -l - 1, c] += 1
    return torch.from_numpy(Ap), torch.from_numpy(An)
