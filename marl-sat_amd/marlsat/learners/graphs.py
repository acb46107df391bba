"""Graph templates + device batch assembly for the GNN encoder.

The reference runs ONE full-size encoder per agent with a masked dense V x C
adjacency (``GNN_ActorCritic.apply_actor``, learner:243-276) plus one unmasked
encoder for the critic (:340-342).  An agent's mask keeps exactly the edges
between its *visible* vars (own vars + vars of clauses touching them) and its
*related* clauses (clauses touching an own var), and every var of a related
clause is visible, so the masked graph's visible/related nodes form a closed
subgraph: their states are identical to the masked full-size computation, and
the other nodes never reach the pooled outputs (learner:287-301).  Hence each
sample is encoded as a ragged batch of small graphs:

  graph 0      critic, all V vars and C clauses
  graph 1 + i  agent i, vars = own (in order) ++ neighbours (ascending), clauses = related (ascending)

Templates are built once per (problem pool, agent partition) on the host (static
data preparation, like packing the pool) and uploaded; per micro-batch a HIP
kernel instantiates them for the sampled (instance, assignment) pairs.  The
adjacency used here is the network's (``create_static_graph``, literal 0 adds
nothing), not the env's literal-0 quirk.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np
import torch

from .. import _lib

# MARLSAT_DEBUG=1: host-side consistency checks that cost a device -> host read (planned vs actual totals)
DEBUG_CHECKS = os.environ.get("MARLSAT_DEBUG") == "1"


def _agent_of(v, base, rem):
    split = rem * (base + 1)
    return np.where(v < split, v // (base + 1), rem + (v - split) // max(base, 1))


def instance_graphs(clauses: np.ndarray, V: int, A: int):
    """Graphs of one instance: list of (var_ids, clause_ids) for g = 0..A."""
    C, K = clauses.shape
    base, rem = divmod(V, A)
    vid = np.abs(clauses).astype(np.int64) - 1
    real = clauses != 0
    ag = np.where(real, _agent_of(np.maximum(vid, 0), base, rem), -1)
    graphs = [(np.arange(V), np.arange(C))]
    for i in range(A):
        lo = i * base + min(i, rem)
        n = base + (1 if i < rem else 0)
        own = np.arange(lo, lo + n)
        rel = np.nonzero((ag == i).any(axis=1))[0]
        vis = np.unique(vid[rel][real[rel]])
        nbr = vis[(vis < lo) | (vis >= lo + n)]
        graphs.append((np.concatenate([own, nbr]), rel))
    return graphs


@dataclass
class Templates:
    """Flattened per-instance templates (host numpy), graph 0 first in every array."""

    vgid: np.ndarray  # (sum vrows,) global var id of each var row
    cgid: np.ndarray  # (sum crows,) global clause id of each clause row
    slots: np.ndarray  # (sum crows, 3) instance-relative (var_row << 1 | neg) or -1
    ptr: np.ndarray  # (sum vrows + N,) per instance: instance-relative CSR pointer (vrows+1 entries)
    inc: np.ndarray  # (sum nnz,) instance-relative (clause_row << 1 | neg)
    voff: np.ndarray  # (N+1,) var-row offset of each instance
    coff: np.ndarray  # (N+1,) clause-row offset
    eoff: np.ndarray  # (N+1,) incidence offset
    poff: np.ndarray  # (N+1,) ptr offset (voff + n)
    gv: np.ndarray  # (N, A+2) graph var-row starts within the instance (cumulative, last = total)
    gc: np.ndarray  # (N, A+2)
    ge: np.ndarray  # (N, A+2) incidence starts per graph


def build_templates(pool_clauses: np.ndarray, V: int, A: int) -> Templates:
    N, C, K = pool_clauses.shape
    vgid, cgid, slots, ptrs, incs = [], [], [], [], []
    voff, coff, eoff, poff = [0], [0], [0], [0]
    gv = np.zeros((N, A + 2), np.int64)
    gc = np.zeros((N, A + 2), np.int64)
    ge = np.zeros((N, A + 2), np.int64)
    for n in range(N):
        cl = pool_clauses[n]
        vid = np.abs(cl).astype(np.int64) - 1
        neg = (cl < 0).astype(np.int64)
        real = cl != 0
        vr, cr = 0, 0
        s_list, v_list, c_list = [], [], []
        for g, (vars_g, cls_g) in enumerate(instance_graphs(cl, V, A)):
            gv[n, g], gc[n, g] = vr, cr
            local = np.full(V, -1, np.int64)
            local[vars_g] = np.arange(len(vars_g)) + vr
            sv = vid[cls_g]
            lv = np.where(real[cls_g], local[np.maximum(sv, 0)], -1)
            assert (lv[real[cls_g]] >= 0).all(), "related clause with an invisible var"
            s = np.where(lv >= 0, (lv << 1) | neg[cls_g], -1)
            if K < 3:
                s = np.concatenate([s, np.full((len(cls_g), 3 - K), -1, np.int64)], 1)
            s_list.append(s)
            v_list.append(vars_g)
            c_list.append(cls_g)
            vr += len(vars_g)
            cr += len(cls_g)
        gv[n, A + 1], gc[n, A + 1] = vr, cr
        s_all = np.concatenate(s_list)  # (crows, 3)
        # var-side CSR (transpose of the slots), entries in (clause row, slot) order
        crow_idx = np.repeat(np.arange(cr), 3)
        flat = s_all.reshape(-1)
        keep = flat >= 0
        vrow = flat[keep] >> 1
        ent = (crow_idx[keep] << 1) | (flat[keep] & 1)
        order = np.argsort(vrow, kind="stable")
        vrow, ent = vrow[order], ent[order]
        counts = np.bincount(vrow, minlength=vr)
        ptr = np.concatenate([[0], np.cumsum(counts)])
        # incidence start of each graph = ptr at its first var row
        for g in range(A + 2):
            ge[n, g] = ptr[gv[n, g]]
        vgid.append(np.concatenate(v_list))
        cgid.append(np.concatenate(c_list))
        slots.append(s_all)
        ptrs.append(ptr)
        incs.append(ent)
        voff.append(voff[-1] + vr)
        coff.append(coff[-1] + cr)
        eoff.append(eoff[-1] + len(ent))
        poff.append(poff[-1] + vr + 1)
    i32 = lambda a: np.asarray(a, np.int32)
    return Templates(i32(np.concatenate(vgid)), i32(np.concatenate(cgid)), i32(np.concatenate(slots)),
                     i32(np.concatenate(ptrs)), i32(np.concatenate(incs)), i32(voff), i32(coff), i32(eoff),
                     i32(poff), i32(gv), i32(gc), i32(ge))


class DeviceTemplates:
    """Templates resident on the device + per-instance totals for batch sizing."""

    def __init__(self, t: Templates, A: int, device):
        dv = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
        self.A, self.G = A, A + 1
        self.vgid, self.cgid, self.slots = dv(t.vgid), dv(t.cgid), dv(t.slots)
        self.ptr, self.inc = dv(t.ptr), dv(t.inc)
        self.voff, self.coff, self.eoff, self.poff = dv(t.voff), dv(t.coff), dv(t.eoff), dv(t.poff)
        self.gv, self.gc, self.ge = dv(t.gv), dv(t.gc), dv(t.ge)
        # rows per instance for a full (critic + agents) sample and for a critic-only sample
        self.full_v = dv(t.gv[:, -1])
        self.full_c = dv(t.gc[:, -1])
        self.full_e = dv(t.ge[:, -1])
        self.crit_v = dv(t.gv[:, 1])
        self.crit_c = dv(t.gc[:, 1])
        self.crit_e = dv(t.ge[:, 1])
        self.max_full_rows = int((t.gv[:, -1] + t.gc[:, -1]).max())
        self.mean_full_rows = float((t.gv[:, -1] + t.gc[:, -1]).mean())


@dataclass
class GraphBatch:
    """Device row-level graph batch of S samples (G graphs each)."""

    S: int
    G: int
    Nv: int
    Nc: int
    nnz: int
    vfeat: torch.Tensor  # (Nv, 8) [x, deg+/C, deg-/C, 0, n+, n-, 0, 0] (n: incidences in the row's graph)
    cfeat: torch.Tensor  # (Nc, 3) [is_sat, ntrue/3, 1]
    cdeg: torch.Tensor  # (Nc, 4) [n+, n-, 0, 0] positive / negative literal slots
    slots: torch.Tensor  # (Nc, 3)
    ptr: torch.Tensor  # (Nv + 1,)
    inc: torch.Tensor  # (nnz,)
    vbase: torch.Tensor  # (S*G,)
    nv: torch.Tensor
    cbase: torch.Tensor
    nc: torch.Tensor


def assemble(tpl: DeviceTemplates, pool_packed: torch.Tensor, svf: torch.Tensor, inst: torch.Tensor,
             x: torch.Tensor, critic_only: bool = False, totals: Optional[Tuple[int, int, int]] = None) -> GraphBatch:
    """Instantiate the templates for samples (inst (S,), x (S,V) uint8) on the device.  ``totals`` =
    the batch's (var rows, clause rows, incidences) when the caller already knows them (the learner
    plans a minibatch's micro-batches at once, batch_totals): no device -> host read here, so the host
    keeps queueing work instead of waiting for the GPU to drain."""
    if totals is not None and critic_only:  # batch_totals plans the full (actor + critic) graphs only
        raise ValueError("assemble: planned totals are for the full graphs; critic_only batches size themselves")
    S = int(inst.shape[0])
    G = 1 if critic_only else tpl.G
    dev = inst.device
    inst = inst.to(torch.int32).contiguous()
    # per-sample row bases (exclusive scans of the instances' row counts) and the batch totals
    sb = torch.empty((max(S, 1), 3), dtype=torch.int32, device=dev)
    tot = torch.empty((3,), dtype=torch.int32, device=dev)
    tv, tc, te = (tpl.crit_v, tpl.crit_c, tpl.crit_e) if critic_only else (tpl.full_v, tpl.full_c, tpl.full_e)
    _lib.check(_lib.lib.msat_graph_bases(S, inst.data_ptr(), tv.data_ptr(), tc.data_ptr(), te.data_ptr(), sb.data_ptr(),
                                         tot.data_ptr(), _lib.stream_ptr(dev)), "msat_graph_bases")
    Nv, Nc, nnz = tot.tolist() if totals is None else totals  # sizes the outputs
    if totals is not None and DEBUG_CHECKS and tuple(tot.tolist()) != tuple(totals):
        raise AssertionError(f"assemble: planned totals {tuple(totals)} != msat_graph_bases {tuple(tot.tolist())}")
    if min(Nv, Nc, nnz) < 0 or max(Nv, Nc, nnz) > 2 ** 31 - 1:  # msat_graph_bases flags an overflow with -1
        raise ValueError(f"graph batch of {S} samples exceeds int32 row indices (var rows, clause rows, incidences "
                         f"= {Nv}, {Nc}, {nnz}; -1 = overflow): use smaller micro-batches")
    # MARLSAT_DEBUG=1: the feature rows start as NaN, so a row the assembly kernel leaves unwritten shows up
    # (libmarlsat_debug.so's GRU backward checks every feature it reads for finiteness)
    feats = (lambda shape: torch.full(shape, float("nan"), device=dev)) if DEBUG_CHECKS else (
        lambda shape: torch.empty(shape, dtype=torch.float32, device=dev))
    out = GraphBatch(S, G, Nv, Nc, nnz, feats((Nv, 8)), feats((Nc, 3)), feats((Nc, 4)),
                     torch.empty((Nc, 3), dtype=torch.int32, device=dev),
                     torch.empty((Nv + 1,), dtype=torch.int32, device=dev),
                     torch.empty((max(nnz, 1),), dtype=torch.int32, device=dev),
                     torch.empty((S * G,), dtype=torch.int32, device=dev),
                     torch.empty((S * G,), dtype=torch.int32, device=dev),
                     torch.empty((S * G,), dtype=torch.int32, device=dev),
                     torch.empty((S * G,), dtype=torch.int32, device=dev))
    V = x.shape[1]
    C = pool_packed.shape[1]
    _lib.check(_lib.lib.msat_assemble_graph_batch(
        S, G, tpl.A, V, C, inst.data_ptr(), x.data_ptr(), svf.data_ptr(), pool_packed.data_ptr(), sb.data_ptr(),
        tpl.vgid.data_ptr(), tpl.cgid.data_ptr(), tpl.slots.data_ptr(), tpl.ptr.data_ptr(), tpl.inc.data_ptr(),
        tpl.voff.data_ptr(), tpl.coff.data_ptr(), tpl.eoff.data_ptr(), tpl.poff.data_ptr(), tpl.gv.data_ptr(),
        tpl.gc.data_ptr(), out.vfeat.data_ptr(), out.cfeat.data_ptr(), out.cdeg.data_ptr(), out.slots.data_ptr(), out.ptr.data_ptr(),
        out.inc.data_ptr(), out.vbase.data_ptr(), out.nv.data_ptr(), out.cbase.data_ptr(), out.nc.data_ptr(),
        Nv, nnz, _lib.stream_ptr(dev)), "msat_assemble_graph_batch")
    return out


def batch_totals(tpl: DeviceTemplates, inst: torch.Tensor, bounds: List[int]) -> List[Tuple[int, int, int]]:
    """(var rows, clause rows, incidences) of the full-sample batches inst[bounds[i]:bounds[i+1]], the
    totals msat_graph_bases computes for each, from ONE device -> host read for all of them
    (int64 sums, so an int32 overflow shows up as a total above INT32_MAX, which assemble refuses)."""
    if len(bounds) < 2:
        return []
    idx = inst.long()
    cnt = torch.stack((tpl.full_v.index_select(0, idx), tpl.full_c.index_select(0, idx),
                       tpl.full_e.index_select(0, idx)), 1).to(torch.int64)
    cs = torch.cat((torch.zeros((1, 3), dtype=torch.int64, device=cnt.device), torch.cumsum(cnt, 0)))
    at = cs.index_select(0, torch.tensor(bounds, dtype=torch.int64, device=cnt.device))
    return [tuple(int(v) for v in r) for r in (at[1:] - at[:-1]).tolist()]
