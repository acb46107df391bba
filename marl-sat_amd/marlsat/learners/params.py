"""Flat parameter layout of the GNN actor-critic + conversion to/from the flax tree.

Device layout (one fp32 buffer, every tensor 16-byte aligned) groups what the
kernels consume together:
  * GRU cells as [ir | iz | in] input matrices (din, 3H), [hr | hz | hn] hidden
    matrices (H, 3H), input bias (3H) and hidden bias [0 | 0 | b_hn] (3H);
  * phi_v_pos / phi_v_neg side by side (H, 2H) — both read H_c;
  * LayerNorm_k as rows [scale | bias] (3L, 2H).
``to_flax`` / ``from_flax`` map it to the reference's flax param names
(GNN_ActorCritic, learner:198-241; encoder :44-80) for checkpoints and parity.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, Tuple

import numpy as np

GATES_I = ("ir", "iz", "in")
GATES_H = ("hr", "hz", "hn")


def layout(H: int, L: int, A: int, M: int, action_mode: int = 0, E: int = 16) -> "OrderedDict[str, Tuple[int, ...]]":
    s: "OrderedDict[str, Tuple[int, ...]]" = OrderedDict()
    for n in ("lpe", "lne", "ce"):
        s[f"enc.{n}_w"] = (3, H)
        s[f"enc.{n}_b"] = (H,)
    s["enc.phi_cp_w"], s["enc.phi_cp_b"] = (H, H), (H,)
    s["enc.phi_cn_w"], s["enc.phi_cn_b"] = (H, H), (H,)
    s["enc.phi_v_w"], s["enc.phi_v_b"] = (H, 2 * H), (2 * H,)
    for cell, din in (("gru_c", 2 * H), ("gru_vp", H + 4), ("gru_vn", H + 4)):
        s[f"enc.{cell}_wi"] = (din, 3 * H)
        s[f"enc.{cell}_bi"] = (3 * H,)
        s[f"enc.{cell}_wh"] = (H, 3 * H)
        s[f"enc.{cell}_bh"] = (3 * H,)
    s["enc.ln"] = (3 * L, 2 * H)
    s["crit.d0_w"], s["crit.d0_b"] = (6 * H, 128), (128,)
    s["crit.d1_w"], s["crit.d1_b"] = (128, 64), (64,)
    s["crit.out_w"], s["crit.out_b"] = (64, 1), (1,)
    s["actor.id_emb"] = (A, E)
    ctx = 5 * H + E
    if action_mode == 0:
        s["actor.flip_d_w"], s["actor.flip_d_b"] = (2 * H + ctx, 128), (128,)
        s["actor.flip_o_w"], s["actor.flip_o_b"] = (128, 1), (1,)
        s["actor.noop_d_w"], s["actor.noop_d_b"] = (ctx, 64), (64,)
        s["actor.noop_o_w"], s["actor.noop_o_b"] = (64, 1), (1,)
    else:
        s["actor.d0_w"], s["actor.d0_b"] = (2 * H + E, 128), (128,)
        s["actor.d1_w"], s["actor.d1_b"] = (128, 64), (64,)
        s["actor.out_w"], s["actor.out_b"] = (64, 2), (2,)
    return s


def offsets(lay) -> Tuple[Dict[str, Tuple[int, Tuple[int, ...]]], int]:
    off, table = 0, {}
    for name, shp in lay.items():
        table[name] = (off, shp)
        n = int(np.prod(shp))
        off += (n + 3) // 4 * 4
    return table, off


_SIMPLE = {  # ours -> flax (kernel, bias)
    "enc.lpe": "encoder/literal_pos_embed", "enc.lne": "encoder/literal_neg_embed",
    "enc.ce": "encoder/clause_embed", "enc.phi_cp": "encoder/phi_c_pos", "enc.phi_cn": "encoder/phi_c_neg",
    "crit.d0": "critic_dense_0", "crit.d1": "critic_dense_1", "crit.out": "critic_output",
    "actor.flip_d": "actor_flip_head_dense", "actor.flip_o": "actor_flip_head_output",
    "actor.noop_d": "actor_noop_head_dense", "actor.noop_o": "actor_noop_head_output",
    "actor.d0": "actor_dense_0", "actor.d1": "actor_dense_1", "actor.out": "actor_output",
}
_CELLS = {"gru_c": "update_c", "gru_vp": "update_v_pos", "gru_vn": "update_v_neg"}


def to_flax(flat: np.ndarray, H: int, L: int, A: int, M: int, action_mode: int = 0, E: int = 16) -> Dict[str, np.ndarray]:
    lay = layout(H, L, A, M, action_mode, E)
    tab, _ = offsets(lay)
    get = lambda n: flat[tab[n][0]: tab[n][0] + int(np.prod(tab[n][1]))].reshape(tab[n][1])
    out = {}
    for ours, fl in _SIMPLE.items():
        if f"{ours}_w" in tab:
            out[f"{fl}/kernel"] = get(f"{ours}_w").copy()
            out[f"{fl}/bias"] = get(f"{ours}_b").copy()
    wv, bv = get("enc.phi_v_w"), get("enc.phi_v_b")
    out["encoder/phi_v_pos/kernel"], out["encoder/phi_v_pos/bias"] = wv[:, :H].copy(), bv[:H].copy()
    out["encoder/phi_v_neg/kernel"], out["encoder/phi_v_neg/bias"] = wv[:, H:].copy(), bv[H:].copy()
    for ours, fl in _CELLS.items():
        wi, bi, wh, bh = (get(f"enc.{ours}_{k}") for k in ("wi", "bi", "wh", "bh"))
        for g, gate in enumerate(GATES_I):
            out[f"encoder/{fl}/{gate}/kernel"] = wi[:, g * H:(g + 1) * H].copy()
            out[f"encoder/{fl}/{gate}/bias"] = bi[g * H:(g + 1) * H].copy()
        for g, gate in enumerate(GATES_H):
            out[f"encoder/{fl}/{gate}/kernel"] = wh[:, g * H:(g + 1) * H].copy()
        out[f"encoder/{fl}/hn/bias"] = bh[2 * H:].copy()
    ln = get("enc.ln")
    for k in range(3 * L):
        out[f"encoder/LayerNorm_{k}/scale"] = ln[k, :H].copy()
        out[f"encoder/LayerNorm_{k}/bias"] = ln[k, H:].copy()
    out["agent_id_embedding/embedding"] = get("actor.id_emb").copy()
    return out


def from_flax(tree: Dict[str, np.ndarray], H: int, L: int, A: int, M: int, action_mode: int = 0,
              E: int = 16) -> np.ndarray:
    lay = layout(H, L, A, M, action_mode, E)
    tab, total = offsets(lay)
    flat = np.zeros(total, np.float32)

    def put(n, v):
        o, shp = tab[n]
        flat[o: o + int(np.prod(shp))] = np.asarray(v, np.float32).reshape(-1)

    for ours, fl in _SIMPLE.items():
        if f"{ours}_w" in tab:
            put(f"{ours}_w", tree[f"{fl}/kernel"])
            put(f"{ours}_b", tree[f"{fl}/bias"])
    put("enc.phi_v_w", np.concatenate([tree["encoder/phi_v_pos/kernel"], tree["encoder/phi_v_neg/kernel"]], 1))
    put("enc.phi_v_b", np.concatenate([tree["encoder/phi_v_pos/bias"], tree["encoder/phi_v_neg/bias"]]))
    for ours, fl in _CELLS.items():
        put(f"enc.{ours}_wi", np.concatenate([tree[f"encoder/{fl}/{g}/kernel"] for g in GATES_I], 1))
        put(f"enc.{ours}_bi", np.concatenate([tree[f"encoder/{fl}/{g}/bias"] for g in GATES_I]))
        put(f"enc.{ours}_wh", np.concatenate([tree[f"encoder/{fl}/{g}/kernel"] for g in GATES_H], 1))
        put(f"enc.{ours}_bh", np.concatenate([np.zeros(2 * H), tree[f"encoder/{fl}/hn/bias"]]))
    put("enc.ln", np.stack([np.concatenate([tree[f"encoder/LayerNorm_{k}/scale"], tree[f"encoder/LayerNorm_{k}/bias"]])
                            for k in range(3 * L)]))
    put("actor.id_emb", tree["agent_id_embedding/embedding"])
    return flat


def init_flat(H: int, L: int, A: int, M: int, action_mode: int = 0, E: int = 16, seed: int = 0) -> np.ndarray:
    """Flax-default init families: lecun-normal kernels (truncated at 2 sd), orthogonal GRU recurrent
    kernels, zero biases, LayerNorm scale 1 / bias 0, Embed normal(1/sqrt(E))."""
    rng = np.random.default_rng(seed)

    def lecun(i, o):
        w = rng.standard_normal((i, o))
        w = np.clip(w, -2, 2) / 0.87962566103423978
        return w / np.sqrt(i)

    def orth(n):
        q, r = np.linalg.qr(rng.standard_normal((n, n)))
        return q * np.sign(np.diag(r))

    tree = {}
    shapes = _flax_shapes(H, L, A, M, action_mode, E)
    for name, shp in shapes.items():
        if name.endswith("/bias"):
            tree[name] = np.zeros(shp)
        elif name.endswith("/scale"):
            tree[name] = np.ones(shp)
        elif name.endswith("/embedding"):
            tree[name] = rng.standard_normal(shp) / np.sqrt(shp[1])
        elif "/h" in name and any(f"/{c}/" in name for c in _CELLS.values()):
            tree[name] = orth(H)
        else:
            tree[name] = lecun(*shp)
    return from_flax(tree, H, L, A, M, action_mode, E)


def _flax_shapes(H, L, A, M, action_mode, E):
    s = {}

    def dense(n, i, o, b=True):
        s[f"{n}/kernel"] = (i, o)
        if b:
            s[f"{n}/bias"] = (o,)

    for n in ("literal_pos_embed", "literal_neg_embed", "clause_embed"):
        dense(f"encoder/{n}", 3, H)
    for n in ("phi_c_pos", "phi_c_neg", "phi_v_pos", "phi_v_neg"):
        dense(f"encoder/{n}", H, H)
    for cell, din in (("update_c", 2 * H), ("update_v_pos", H + 4), ("update_v_neg", H + 4)):
        for g in GATES_I:
            dense(f"encoder/{cell}/{g}", din, H)
        dense(f"encoder/{cell}/hr", H, H, False)
        dense(f"encoder/{cell}/hz", H, H, False)
        dense(f"encoder/{cell}/hn", H, H)
    for k in range(3 * L):
        s[f"encoder/LayerNorm_{k}/scale"] = (H,)
        s[f"encoder/LayerNorm_{k}/bias"] = (H,)
    dense("critic_dense_0", 6 * H, 128)
    dense("critic_dense_1", 128, 64)
    dense("critic_output", 64, 1)
    s["agent_id_embedding/embedding"] = (A, E)
    ctx = 5 * H + E
    if action_mode == 0:
        dense("actor_flip_head_dense", 2 * H + ctx, 128)
        dense("actor_flip_head_output", 128, 1)
        dense("actor_noop_head_dense", ctx, 64)
        dense("actor_noop_head_output", 64, 1)
    else:
        dense("actor_dense_0", 2 * H + E, 128)
        dense("actor_dense_1", 128, 64)
        dense("actor_output", 64, 2)
    return s
