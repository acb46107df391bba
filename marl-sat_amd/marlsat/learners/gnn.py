"""GNN actor-critic on the device: forward, backward and Adam over the HIP kernels.

Mirrors ``GNN_ActorCritic`` (src/learners/mappo_gnn_sat_learner.py:198-355) and
``GNNEncoder`` (:19-82) on a ragged graph batch (graphs.py).  Every matmul is the
fp32 MFMA GEMM of gemm.hip, the message passing is the signed literal gathers,
GRU + LayerNorm and the heads are fused kernels; torch only allocates memory.

Per message step l the forward keeps, for the backward pass, the step inputs
(Hp, Hn, Hc), the gathered clause input, the var-side messages and the six GRU
gate pre-activations; the backward walks the steps in reverse, accumulating
every weight gradient through the split-M weight-gradient GEMM (fixed reduction
order: the whole update is bitwise reproducible).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch

from .. import _lib
from . import params as P
from .graphs import GraphBatch

L_ = _lib.lib

# Arithmetic of the matrix work (README "Kernel-path switches"): "fp16x2" (default) runs the GRU
# forward and the backward's data / weight gradients on fp16 MFMAs with a two-way fp32 split, falling
# back per tile to "bf16x3" (three-way bf16 split) where fp16's range fails; "bf16x3" runs that
# fallback throughout; "fp32" keeps every product on fp32 MFMA (the accuracy reference path).
PRECISION = os.environ.get("MARLSAT_PRECISION", "fp16x2")
PRECISION_CODES = {"fp16x2": 0, "bf16x3": 1, "fp32": 2}  # MSAT_PRECISION_* (include/marlsat_net.h)
if PRECISION not in PRECISION_CODES:
    raise ValueError(f"MARLSAT_PRECISION must be fp16x2, bf16x3 or fp32, got {PRECISION!r}")
# the library's weight-gradient path follows the same validated value (set once, not re-read per call)
_lib.check(L_.msat_set_precision(PRECISION_CODES[PRECISION]), "msat_set_precision")


def _chk(rc, what):
    if rc:
        _lib.check(rc, what)


class _Scratch:
    """Grow-only device scratch (ones vector, wgrad workspace, LN partials)."""

    def __init__(self, device):
        self.device = device
        self.ones = torch.ones(1, device=device)
        self.ws = torch.empty(1, device=device)
        self.part = torch.empty(1, device=device)

    def get_ones(self, n):
        if self.ones.numel() < n:
            self.ones = torch.ones(max(n, 2 * self.ones.numel()), device=self.device)
        return self.ones

    def get_ws(self, nbytes):
        n = (nbytes + 3) // 4 + 1
        if self.ws.numel() < n:
            self.ws = torch.empty(max(n, 2 * self.ws.numel()), device=self.device)
        return self.ws

    def get_flags(self, n):
        if getattr(self, "flags", None) is None or self.flags.numel() < n:
            self.flags = torch.empty(max(n, 1024), dtype=torch.int32, device=self.device)
        return self.flags

    def get_part(self, n):
        if self.part.numel() < n:
            self.part = torch.empty(max(n, 2 * self.part.numel()), device=self.device)
        return self.part


@dataclass
class StepTape:
    Hp: torch.Tensor
    Hn: torch.Tensor
    Hc: torch.Tensor
    GIN: torch.Tensor  # (Nc, 2H) clause GRU input: gathered [sum H_v+ | sum H_v-] (fused) or messages (ref)
    G4c: torch.Tensor  # (Nc, 4H) clause GRU pre-activations [r | z | gin | ghn]
    NV: torch.Tensor  # (Nv, 2H) var GRU inputs: gathered [sum H_c over + | over -] (fused) or messages (ref)
    G4p: torch.Tensor  # (Nv, 4H) update_v_pos pre-activations
    G4n: torch.Tensor  # (Nv, 4H) update_v_neg pre-activations


@dataclass
class HeadTape:
    pooled: Optional[torch.Tensor] = None
    c0: Optional[torch.Tensor] = None
    c1: Optional[torch.Tensor] = None
    my: Optional[torch.Tensor] = None
    ctx: Optional[torch.Tensor] = None
    h1: Optional[torch.Tensor] = None
    n1: Optional[torch.Tensor] = None
    h2: Optional[torch.Tensor] = None  # mode 1 second hidden layer


class GNNActorCritic:
    """Device GNN_ActorCritic with flat parameters (params.py layout)."""

    def __init__(self, gnn_hidden_dim: int, gnn_num_message_passing_steps: int, num_agents: int,
                 max_vars_per_agent: int, action_mode: int, num_vars: int, agent_id_embed_dim: int = 16,
                 device=None, seed: int = 0):
        self.H, self.L = gnn_hidden_dim, gnn_num_message_passing_steps
        self.A, self.M, self.mode, self.E = num_agents, max_vars_per_agent, action_mode, agent_id_embed_dim
        self.V = num_vars
        self.base, self.rem = divmod(num_vars, num_agents)
        self.CW = 5 * self.H + self.E
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.layout = P.layout(self.H, self.L, self.A, self.M, self.mode, self.E)
        self.tab, self.size = P.offsets(self.layout)
        self.params = torch.from_numpy(P.init_flat(self.H, self.L, self.A, self.M, self.mode, self.E, seed)).to(self.device)
        self.grads = torch.zeros_like(self.params)
        self.adam_m = torch.zeros_like(self.params)
        self.adam_v = torch.zeros_like(self.params)
        self.adam_count = 0
        self.scr = _Scratch(self.device)

    # ----------------------------------------------------------- plumbing ----
    def load_flax(self, tree):
        self.params.copy_(torch.from_numpy(P.from_flax(tree, self.H, self.L, self.A, self.M, self.mode, self.E)))

    def to_flax(self, grads: bool = False):
        t = (self.grads if grads else self.params).detach().cpu().numpy()
        return P.to_flax(t, self.H, self.L, self.A, self.M, self.mode, self.E)

    def p(self, name: str) -> torch.Tensor:
        o, shp = self.tab[name]
        return self.params[o: o + int(np.prod(shp))].view(shp)

    def g(self, name: str) -> torch.Tensor:
        o, shp = self.tab[name]
        return self.grads[o: o + int(np.prod(shp))].view(shp)

    @property
    def stream(self):
        return _lib.stream_ptr(self.device)

    flops = 0  # matmul FLOPs issued (2*M*N*K per GEMM), for the MFMA roofline

    # bench.py's per-kernel roofline: a dict makes the MFMA kernels' launches record
    # {label: [(start event, end event, fp32-equivalent algorithmic FLOPs)]} on the launch stream
    ktimer: Optional[dict] = None

    def _timed(self, label: str, flop: float, call, nbytes: float = 0.0):
        """Run `call`; under bench.py's ktimer record (start, end, algorithmic fp32 FLOPs, algorithmic HBM
        bytes: operands read once + results written, no re-reads or workspaces)."""
        kt = GNNActorCritic.ktimer
        if kt is None:
            return call()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = call()
        e1.record()
        kt.setdefault(label, []).append((e0, e1, float(flop), float(nbytes)))
        return r

    @staticmethod
    def _span(p0: int, p1: int, width: int, ld: int) -> int:
        """Floats per row read by two row windows [p, p + width) (byte pointers) of one row-major buffer
        with ld floats per row: their union if they overlap within a row, else both."""
        lo, hi = min(p0, p1), max(p0, p1) + 4 * width
        return (hi - lo) // 4 if hi - lo <= 4 * ld else 2 * width

    def _gemm(self, A, lda, B, ldb, transB, C, ldc, bias, M, N, K, acc=0):
        GNNActorCritic.flops += 2 * M * N * K
        self._timed("msat_gemm (fp32 MFMA)", 2.0 * M * N * K, lambda: _chk(
            L_.msat_gemm(A, lda, B, ldb, transB, C, ldc, bias, M, N, K, acc, self.stream), "msat_gemm"),
            4.0 * (M * K + N * K + M * N * (1 + acc)))

    def _gemm64(self, A, lda, transA, B, ldb, transB, C, ldc, M, N, K, acc=0):
        """fp64-accumulated small product, one rounding per element (the folded weights, gemm.hip)."""
        _chk(L_.msat_gemm_f64acc(A, lda, transA, B, ldb, transB, C, ldc, M, N, K, acc, self.stream),
             "msat_gemm_f64acc")

    # fp32-accurate bf16x3 split GEMM for the backward's C (+)= dG @ W^T products (gemm_x3.hip)
    use_x3 = PRECISION != "fp32"

    def _split_weights(self, mats):
        """bf16x3 planes of each (rows, 3H) weight block (once per backward): {key: planes tensor}.
        mats: {key: (matrix, column rotation)}; rotation 2H puts the gate blocks in (n, r, z) order,
        the order of the packed backward rows' dGi columns."""
        out = {}
        for key, (Wm, rot) in mats.items():
            rows, cols = Wm.shape
            buf = torch.empty(3 * rows * cols + 8, dtype=torch.int16, device=self.device)
            _chk(L_.msat_split_bf16x3_rot(Wm.data_ptr(), rows, cols, cols, rot, buf.data_ptr(), self.stream),
                 "split_bf16x3")
            out[key] = buf
        return out

    # fp16x2 data gradients of the packed backward rows (gemm_x3.hip gemm_h2r16_kernel)
    use_dgrad_h2 = PRECISION == "fp16x2"

    # a cell's two data gradients / two weight gradients in one launch each (gemm_x3.hip *_dual_kernel;
    # the fp16x2 path always takes them: -4 % against separate launches, round 2)
    use_dual = True

    # the packed backward rows as fp16x2 planes (gnn_kernels.hip flags bit 3): split once per row in the GRU
    # backward instead of once per consumer and k tile; the dual products read the planes (round 5)
    use_planes = os.environ.get("MARLSAT_PLANES", "1") != "0"

    def _dgrad_dual(self, p0, p1, rexp, M, K, pbase=None):
        """p = (A, lda, fp16x2 planes, bf16x3 planes, wbad pointer, C, ldc, N, accumulate): both
        C (+)= A @ W^T products over the same M rows (row exponents rexp) in one fp16x2 launch.  pbase: the
        packed buffer's base when it holds fp16x2 planes (A pointers are then its fp32 column addresses)."""
        if M == 0:
            return
        fl = 2.0 * M * K * (p0[7] + p1[7])
        GNNActorCritic.flops += fl
        nb = 4.0 * M * (self._span(p0[0], p1[0], K, p0[1]) + p0[7] * (1 + p0[8]) + p1[7] * (1 + p1[8]) + 1)
        if pbase is not None:  # fp32 column c of a packed row -> its hi-plane element c (same bytes per row)
            pa = lambda p: pbase + (p[0] - pbase) // 2
            self._timed("gemm_h2r16_kernel (dgrad, fp16x2 planes)", fl, lambda: _chk(L_.msat_gemm_h2_dual_planes(
                pa(p0), 2 * p0[1], p0[2].data_ptr(), p0[3].data_ptr(), p0[4], p0[5], p0[6], p0[7], p0[8],
                pa(p1), 2 * p1[1], p1[2].data_ptr(), p1[3].data_ptr(), p1[4], p1[5], p1[6], p1[7], p1[8],
                p0[1], rexp.data_ptr(), M, K, self.stream), "msat_gemm_h2_dual_planes"), nb)
            return
        self._timed("gemm_h2r16_kernel (dgrad, fp16x2)", fl, lambda: _chk(L_.msat_gemm_h2_dual(
            p0[0], p0[1], p0[2].data_ptr(), p0[3].data_ptr(), p0[4], p0[5], p0[6], p0[7], p0[8],
            p1[0], p1[1], p1[2].data_ptr(), p1[3].data_ptr(), p1[4], p1[5], p1[6], p1[7], p1[8],
            rexp.data_ptr(), M, K, self.stream), "msat_gemm_h2_dual"), nb)

    def _wgrad_h2_dual(self, p0, p1, rexp, M, acc=1, pbase=None):
        """p = (A, lda, G, ldg, W, ldw, K, N, rot): both W[:, (n + rot) % N] (+)= (A^T G)[:, n] over the same M
        rows of G's buffer (row exponents rexp) in one fp16x2 launch.  pbase: as _dgrad_dual (G's buffer holds
        fp16x2 planes)."""
        if M == 0:
            return
        fl = 2.0 * M * (p0[6] * p0[7] + p1[6] * p1[7])
        GNNActorCritic.flops += fl
        ws = self.scr.get_ws(int(L_.msat_gemm_wgrad_dual_workspace_bytes(M, p0[6], p0[7], p1[6], p1[7])))
        nb = 4.0 * M * (p0[6] + p1[6] + self._span(p0[2], p1[2], p0[7], p0[3]) + 1)  # A rows, G rows, rexp
        if pbase is not None:
            pg = lambda p: p[:2] + (pbase + (p[2] - pbase) // 2, 2 * p[3]) + p[4:]
            self._timed("wgrad_w_dual_pl_kernel + fixup + reduce (fp16x2 planes)", fl, lambda: _chk(
                L_.msat_gemm_wgrad_h2_dual_planes(*pg(p0), *pg(p1), p0[3], rexp.data_ptr(), M, acc, ws.data_ptr(),
                                                  self.stream), "msat_gemm_wgrad_h2_dual_planes"), nb)
            return
        self._timed("wgrad_w_kernel<2> + fixup + reduce (fp16x2)", fl, lambda: _chk(L_.msat_gemm_wgrad_h2_dual(
            *p0, *p1, rexp.data_ptr(), M, acc, ws.data_ptr(), self.stream), "msat_gemm_wgrad_h2_dual"), nb)

    def _split_weights_f16(self, mats):
        """fp16x2 planes (2^10 W, msat_split_f16x2_rot) of each block of `mats` (as _split_weights):
        ({key: planes tensor}, {key: wbad pointer}); wbad[key] = 1 if the block overflowed fp16."""
        bad = torch.empty(len(mats), dtype=torch.int32, device=self.device)
        out, bp = {}, {}
        for i, (key, (Wm, rot)) in enumerate(mats.items()):
            rows, cols = Wm.shape
            buf = torch.empty(2 * rows * cols + 8, dtype=torch.int16, device=self.device)
            _chk(L_.msat_split_f16x2_rot(Wm.data_ptr(), rows, cols, cols, rot, buf.data_ptr(), self._ptr(bad, i),
                                         self.stream), "split_f16x2_rot")
            out[key], bp[key] = buf, self._ptr(bad, i)
        out["_bad"] = bad  # keep-alive
        return out, bp

    def _dgrad(self, A, lda, Wm: torch.Tensor, planes, C, ldc, M, N, K, acc, h2=None):
        """C[M,N] (+)= A[M,K] @ Wm[:N]^T (Wm rows = N, row stride K).  h2 = (fp16x2 planes, wbad pointer,
        A's row exponents): the fp16x2 kernel (its bf16x3 body on `planes` if the split overflowed)."""
        if h2 is not None and M > 0:
            p2, wbad, rexp = h2
            GNNActorCritic.flops += 2 * M * N * K
            self._timed("gemm_h2r16_kernel (dgrad, fp16x2)", 2.0 * M * N * K, lambda: _chk(
                L_.msat_gemm_h2(A, lda, rexp.data_ptr(), p2.data_ptr(), planes.data_ptr(), wbad, C, ldc, None, M, N,
                                K, acc, self.stream), "msat_gemm_h2"), 4.0 * M * (K + N * (1 + acc) + 1))
            return
        if planes is None:
            self._gemm(A, lda, Wm.data_ptr(), K, 1, C, ldc, None, M, N, K, acc)
            return
        GNNActorCritic.flops += 2 * M * N * K
        self._timed("gemm_x3r16_kernel (dgrad, bf16x3)", 2.0 * M * N * K, lambda: _chk(
            L_.msat_gemm_x3(A, lda, planes.data_ptr(), C, ldc, None, M, N, K, acc, self.stream), "msat_gemm_x3"),
            4.0 * M * (K + N * (1 + acc)))

    def _wgrad(self, A, lda, G, ldg, W, ldw, M, K, N, acc=1, rot=0):
        """W[:, (n + rot) % N] (+)= (A^T G)[:, n] (rot: the packed rows' gate-block rotation)."""
        if M == 0:
            return
        GNNActorCritic.flops += 2 * M * N * K
        ws = self.scr.get_ws(int(L_.msat_gemm_wgrad_workspace_bytes(M, K, N)))
        if K <= 8:
            label = "wgrad_skinny + reduce (K <= 8)"
        elif N <= 384:
            label = "wgrad_w_kernel<3> + reduce (bf16x3)"
        else:
            label = "wgrad_x3_kernel + reduce (bf16x3)"
        self._timed(label, 2.0 * M * N * K, lambda: _chk(
            L_.msat_gemm_wgrad_rot(A, lda, G, ldg, W, ldw, M, K, N, rot, acc, ws.data_ptr(), self.stream),
            "msat_gemm_wgrad_rot"), 4.0 * M * (K + N))

    # fp16x2 whole-row weight gradients of the GRU backward's packed rows (gemm_x3.hip wgrad_w_kernel<2>):
    # the backward writes each row's scale exponent, the kernel scales G per row split
    use_wgrad_h2 = PRECISION == "fp16x2"

    def _wgrad_h2(self, A, lda, G, ldg, rexp, W, ldw, M, K, N, acc=1, rot=0):
        """W[:, (n + rot) % N] (+)= (A^T G)[:, n] in fp16x2; rexp: G's row scale exponents."""
        if M == 0:
            return
        GNNActorCritic.flops += 2 * M * N * K
        ws = self.scr.get_ws(int(L_.msat_gemm_wgrad_workspace_bytes(M, K, N)))
        self._timed("wgrad_w_kernel<2> + fixup + reduce (fp16x2)", 2.0 * M * N * K, lambda: _chk(
            L_.msat_gemm_wgrad_h2(A, lda, G, ldg, rexp.data_ptr(), W, ldw, M, K, N, rot, acc, ws.data_ptr(),
                                  self.stream),
            "msat_gemm_wgrad_h2"), 4.0 * M * (K + N + 1))

    def _colsum(self, G, ldg, M, N, out, acc=1):
        if M == 0:
            return
        ws = self.scr.get_part(int(L_.msat_colsum_workspace_floats(M, N)))
        _chk(L_.msat_colsum(G, ldg, M, N, out, acc, ws.data_ptr(), self.stream), "msat_colsum")

    # split GRU kernels (fp32-accurate, 16x16x32 MFMAs, register-A) for the fused encoder at H = 128:
    # bf16x3 (gru_fused.hip x3r), and the fp16x2 kernel below with x3r as its fixup; else fp32 MFMA
    use_gru_x3 = PRECISION != "fp32"

    def _split_weights_t(self, mats):
        """{key: (K, 3H) matrix} -> {key: (W^T bf16x3 planes (3, 3H, Kp), Kp)}, Kp = K rounded up to 32
        (msat_split_bf16x3_t: transposed, zero-padded, split in one pass; once per forward)."""
        out = {}
        for key, Wm in mats.items():
            K, N = Wm.shape
            Kp = (K + 31) // 32 * 32
            buf = torch.empty(3 * N * Kp + 8, dtype=torch.int16, device=self.device)
            _chk(L_.msat_split_bf16x3_t(Wm.data_ptr(), K, N, Wm.stride(0), Kp, buf.data_ptr(), self.stream),
                 "split_bf16x3_t")
            out[key] = (buf, Kp)
        return out

    # fp16x2 operands for the register-A GRU forward (gru_fused.hip kRH2: three fp16 MFMAs per product
    # instead of six bf16 ones, two weight planes instead of three; tiles whose activations leave fp16's
    # range are recomputed in bf16x3 by the same launch pair); MARLSAT_GRU_H2=0 keeps bf16x3 throughout
    use_gru_h2 = PRECISION == "fp16x2"

    def _split_weights_h2(self, cells):
        """{cell: (Wi (Kx, 3H), Wh (H, 3H))} -> ({cell: (wi planes, wh planes)}, wbad (cells, 2) int32):
        the transposed fp16x2 planes (msat_split_f16x2_t, weights scaled by 2^10) of both matrices of each
        cell; wbad[c] = [wi overflowed, wh overflowed] (device flags read by the GRU launch)."""
        bad = torch.empty((len(cells), 2), dtype=torch.int32, device=self.device)
        out = {}
        for c, (key, mats) in enumerate(cells.items()):
            bufs = []
            for m, Wm in enumerate(mats):
                K, N = Wm.shape
                Kp = (K + 31) // 32 * 32
                buf = torch.empty(2 * N * Kp + 8, dtype=torch.int16, device=self.device)
                _chk(L_.msat_split_f16x2_t(Wm.data_ptr(), K, N, Wm.stride(0), Kp, buf.data_ptr(),
                                           self._ptr(bad[c], m), self.stream), "split_f16x2_t")
                bufs.append(buf)
            out[key] = (bufs[0], bufs[1], self._ptr(bad[c]))
        return out, bad

    def _gru(self, cell: str, segs, hprev: torch.Tensor, ln_row: torch.Tensor, out: torch.Tensor,
             g4: Optional[torch.Tensor], R: int, wi: Optional[torch.Tensor] = None, wt=None):
        """One fused GRU cell + LayerNorm (msat_gru_ln_fused_fwd): segs = [(ptr, ld, width)] of x;
        wi overrides the cell's input matrix (the phi-folded matrices of the fused encoder);
        wt = {"wi": (W^T planes, kxp), "wh": planes[, "h2": fp16x2 planes]} selects the register-A
        bf16x3 kernel (msat_gru_ln_fused_fwd_x3r) or, with "h2", the fp16x2 one + its bf16x3 fixup."""
        H = self.H
        segs = list(segs) + [(0, 0, 0)] * (3 - len(segs))
        kx = sum(w for _, _, w in segs)
        GNNActorCritic.flops += 2 * R * 3 * H * (H + (kx + 15) // 16 * 16)
        (p0, l0, w0), (p1, l1, w1), (p2, l2, w2) = segs
        if isinstance(wt, dict) and wt.get("h2"):  # fp16x2 register-A kernel + bf16x3 fixup of flagged tiles
            h2wi, h2wh, wbad = wt["h2"]
            flags = self.scr.get_flags((R + 127) // 128)
            nb = 4.0 * R * (kx + 2 * H + (4 * H if g4 is not None else 0))  # x, h in; h' (+ tape) out
            self._timed("gru_ln_fused_fwd_h2s_kernel (fp16x2, + x3r fixup launch)", 2.0 * R * 3 * H * (H + kx), lambda: _chk(
                L_.msat_gru_ln_fused_fwd_h2r(p0, l0, w0, p1, l1, w1, p2, l2, w2, hprev.data_ptr(), H,
                                             h2wi.data_ptr(), h2wh.data_ptr(), wt["wi"][0].data_ptr(),
                                             wt["wh"].data_ptr(), wt["wi"][1], self.p(f"enc.{cell}_bi").data_ptr(),
                                             self.p(f"enc.{cell}_bh").data_ptr(), self._ptr(ln_row),
                                             self._ptr(ln_row, H), out.data_ptr(), H,
                                             g4.data_ptr() if g4 is not None else 0, 4 * H, R, H, flags.data_ptr(),
                                             wbad, self.stream),
                "msat_gru_ln_fused_fwd_h2r"), nb)
            return
        if isinstance(wt, dict):  # register-A bf16x3 kernel: W^T planes {"wi": (planes, kxp), "wh": planes}
            self._timed("gru_ln_fused_fwd_x3r_kernel (bf16x3)", 2.0 * R * 3 * H * (H + kx), lambda: _chk(
                L_.msat_gru_ln_fused_fwd_x3r(p0, l0, w0, p1, l1, w1, p2, l2, w2, hprev.data_ptr(), H,
                                             wt["wi"][0].data_ptr(), wt["wi"][1],
                                             self.p(f"enc.{cell}_bi").data_ptr(), wt["wh"].data_ptr(),
                                             self.p(f"enc.{cell}_bh").data_ptr(), self._ptr(ln_row),
                                             self._ptr(ln_row, H), out.data_ptr(), H,
                                             g4.data_ptr() if g4 is not None else 0, 4 * H, R, H, self.stream),
                "msat_gru_ln_fused_fwd_x3r"), 4.0 * R * (kx + 2 * H + (4 * H if g4 is not None else 0)))
            return
        _chk(L_.msat_gru_ln_fused_fwd(p0, l0, w0, p1, l1, w1, p2, l2, w2, hprev.data_ptr(), H,
                                      (self.p(f"enc.{cell}_wi") if wi is None else wi).data_ptr(),
                                      self.p(f"enc.{cell}_bi").data_ptr(),
                                      self.p(f"enc.{cell}_wh").data_ptr(), self.p(f"enc.{cell}_bh").data_ptr(),
                                      self._ptr(ln_row), self._ptr(ln_row, H), out.data_ptr(), H,
                                      g4.data_ptr() if g4 is not None else 0, 4 * H, R, H, self.stream),
             "msat_gru_ln_fused_fwd")

    @staticmethod
    def _ptr(t: torch.Tensor, col: int = 0) -> int:
        return t.data_ptr() + col * t.element_size()

    # ---------------------------------------------------------- encoder ----
    def encode(self, b: GraphBatch, save: bool):
        return self._encode_fused(b, save) if self.fuse_phi else self._encode_ref(b, save)

    def encode_backward(self, b: GraphBatch, tape: List[StepTape], Hc_final, dHp, dHn, dHc):
        if self.fuse_phi:
            self._encode_backward_fused(b, tape, Hc_final, dHp, dHn, dHc)
        else:
            self._encode_backward_ref(b, tape, Hc_final, dHp, dHn, dHc)

    def _embed(self, b: GraphBatch):
        """literal / clause embeddings (learner:57-59): vfeat[:, 1:4] = svf, cfeat = clause features."""
        H, e = self.H, lambda *shape: torch.empty(shape, dtype=torch.float32, device=self.device)
        pp = self._ptr
        Hp, Hn, Hc = e(b.Nv, H), e(b.Nv, H), e(b.Nc, H)
        self._gemm(pp(b.vfeat, 1), 8, self.p("enc.lpe_w").data_ptr(), H, 0, Hp.data_ptr(), H,
                   self.p("enc.lpe_b").data_ptr(), b.Nv, H, 3)
        self._gemm(pp(b.vfeat, 1), 8, self.p("enc.lne_w").data_ptr(), H, 0, Hn.data_ptr(), H,
                   self.p("enc.lne_b").data_ptr(), b.Nv, H, 3)
        self._gemm(b.cfeat.data_ptr(), 3, self.p("enc.ce_w").data_ptr(), H, 0, Hc.data_ptr(), H,
                   self.p("enc.ce_b").data_ptr(), b.Nc, H, 3)
        return Hp, Hn, Hc

    def _embed_backward(self, b: GraphBatch, dHp, dHn, dHc):
        H, pp = self.H, self._ptr
        Nv, Nc = b.Nv, b.Nc
        self._wgrad(pp(b.vfeat, 1), 8, dHp.data_ptr(), H, self.g("enc.lpe_w").data_ptr(), H, Nv, 3, H)
        self._colsum(dHp.data_ptr(), H, Nv, H, self.g("enc.lpe_b").data_ptr())
        self._wgrad(pp(b.vfeat, 1), 8, dHn.data_ptr(), H, self.g("enc.lne_w").data_ptr(), H, Nv, 3, H)
        self._colsum(dHn.data_ptr(), H, Nv, H, self.g("enc.lne_b").data_ptr())
        self._wgrad(b.cfeat.data_ptr(), 3, dHc.data_ptr(), H, self.g("enc.ce_w").data_ptr(), H, Nc, 3, H)
        self._colsum(dHc.data_ptr(), H, Nc, H, self.g("enc.ce_b").data_ptr())

    # Fused encoder ("gather first, phi folded into the GRU input matrix").  Per message step
    # the reference computes m_c+ = A+^T (H_v+ Wcp + bcp) and feeds [m_c+ | m_c-] through
    # update_c's input matrix Wi_c (learner:66-69); by linearity
    #     [m_c+ | m_c-] Wi_c = [A+^T H_v+ | A-^T H_v-] [[Wcp Wi_c+], [Wcn Wi_c-]] + n+ (bcp Wi_c+) + n- (bcn Wi_c-)
    # with n+/- the clause row's positive / negative slot counts, and likewise on the var side
    # n_v+ Wi_vp,n = (A+ H_c)(Wv+ Wi_vp,n) + deg+ (bv+ Wi_vp,n)  (learner:72-79).  So each step
    # is two gathers of the node STATES plus the three fused GRU kernels, with the folded
    # matrices F (rows: [products | count-column rows]) rebuilt once per forward; the phi GEMMs
    # (forward, input-gradient and weight-gradient) disappear and the weight gradients of
    # phi / Wi are recovered from dF once per backward (_unfuse_grads).  Same function,
    # different fp32 association: parity is the 1e-5 fp32 bar, not bitwise.
    # the fp32 path is the reference's operation order: phi stays unfolded there unless MARLSAT_FUSE_PHI says so
    fuse_phi = os.environ.get("MARLSAT_FUSE_PHI", "0" if PRECISION == "fp32" else "1") != "0"

    def _fold_views(self):
        """Views of the folded matrices F_c (2H+4 rows), F_v+, F_v- (H+8 rows) and of their gradients
        (each block 16-row aligned in one buffer, zero rows between)."""
        H = self.H
        c, v = 2 * H + 4, H + 8
        cp, vp = (c + 15) // 16 * 16, (v + 15) // 16 * 16
        if getattr(self, "_F", None) is None:
            self._F = torch.zeros((cp + 2 * vp, 3 * H), dtype=torch.float32, device=self.device)
            self._gF = torch.zeros_like(self._F)
        sl = lambda T: (T[:c], T[cp:cp + v], T[cp + vp:cp + vp + v])
        return sl(self._F), sl(self._gF)

    def _fold_weights(self):
        """F_c (2H+4, 3H) = [Wcp Wi_c[:H]; Wcn Wi_c[H:]; bcp Wi_c[:H]; bcn Wi_c[H:]; 0; 0]
        F_v+ (H+8, 3H) = [Wv+ Wi_vp[:H]; Wi_vp[H:H+4]; bv+ Wi_vp[:H]; 0; 0; 0]
        F_v- (H+8, 3H) = [Wv- Wi_vn[:H]; Wi_vn[H:H+4]; 0; bv- Wi_vn[:H]; 0; 0]  (pad rows stay 0)."""
        H, pp = self.H, self._ptr
        (Fc, Fp, Fn), _ = self._fold_views()
        W3 = 3 * H
        wic = self.p("enc.gru_c_wi")
        # F multiplies every row of every step: computed in fp64 and rounded once (a plain fp32 product's
        # rounding is a systematic weight error that 16 GRU + LayerNorm steps accumulate coherently)
        for half, nm in ((0, "phi_cp"), (1, "phi_cn")):
            B = pp(wic[half * H])
            self._gemm64(self.p(f"enc.{nm}_w").data_ptr(), H, 0, B, W3, 0, pp(Fc[half * H]), W3, H, W3, H)
            self._gemm64(self.p(f"enc.{nm}_b").data_ptr(), H, 0, B, W3, 0, pp(Fc[2 * H + half]), W3, 1, W3, H)
        wv, bv = self.p("enc.phi_v_w"), self.p("enc.phi_v_b")
        for half, cell, F in ((0, "gru_vp", Fp), (1, "gru_vn", Fn)):
            wi = self.p(f"enc.{cell}_wi")
            self._gemm64(pp(wv, half * H), 2 * H, 0, wi.data_ptr(), W3, 0, F.data_ptr(), W3, H, W3, H)
            F[H:H + 4].copy_(wi[H:H + 4])
            self._gemm64(pp(bv, half * H), H, 0, wi.data_ptr(), W3, 0, pp(F[H + 4 + half]), W3, 1, W3, H)

    def _unfuse_grads(self):
        """dF -> phi / Wi gradients (F = W Wi: dW = dF Wi^T, dWi = W^T dF; bias rows likewise)."""
        H, pp = self.H, self._ptr
        _, (gFc, gFp, gFn) = self._fold_views()
        W3 = 3 * H
        wic, gwic = self.p("enc.gru_c_wi"), self.g("enc.gru_c_wi")
        for half, nm in ((0, "phi_cp"), (1, "phi_cn")):
            B, gB = pp(wic[half * H]), pp(gwic[half * H])
            self._gemm64(pp(gFc[half * H]), W3, 0, B, W3, 1, self.g(f"enc.{nm}_w").data_ptr(), H, H, H, W3, 1)
            self._gemm64(pp(gFc[2 * H + half]), W3, 0, B, W3, 1, self.g(f"enc.{nm}_b").data_ptr(), H, 1, H, W3, 1)
            self._gemm64(self.p(f"enc.{nm}_w").data_ptr(), H, 1, pp(gFc[half * H]), W3, 0, gB, W3, H, W3, H, 1)
            self._gemm64(self.p(f"enc.{nm}_b").data_ptr(), H, 1, pp(gFc[2 * H + half]), W3, 0, gB, W3, H, W3, 1, 1)
        wv, bv = self.p("enc.phi_v_w"), self.p("enc.phi_v_b")
        gwv, gbv = self.g("enc.phi_v_w"), self.g("enc.phi_v_b")
        for half, cell, gF in ((0, "gru_vp", gFp), (1, "gru_vn", gFn)):
            wi, gwi = self.p(f"enc.{cell}_wi"), self.g(f"enc.{cell}_wi")
            self._gemm64(gF.data_ptr(), W3, 0, wi.data_ptr(), W3, 1, pp(gwv, half * H), 2 * H, H, H, W3, 1)
            self._gemm64(pp(gF[H + 4 + half]), W3, 0, wi.data_ptr(), W3, 1, pp(gbv, half * H), H, 1, H, W3, 1)
            self._gemm64(pp(wv, half * H), 2 * H, 1, gF.data_ptr(), W3, 0, gwi.data_ptr(), W3, H, W3, H, 1)
            self._gemm64(pp(bv, half * H), H, 1, pp(gF[H + 4 + half]), W3, 0, gwi.data_ptr(), W3, H, W3, 1, 1)
            self._colsum(pp(gF[H]), 4 * W3, 1, 4 * W3, pp(gwi[H]))  # the x / svf rows map 1:1

    def _encode_fused(self, b: GraphBatch, save: bool):
        H, dev = self.H, self.device
        Nv, Nc = b.Nv, b.Nc
        e = lambda *shape: torch.empty(shape, dtype=torch.float32, device=dev)
        pp = self._ptr
        self._fold_weights()
        (Fc, Fp, Fn), _ = self._fold_views()
        wt = {"gru_c": None, "gru_vp": None, "gru_vn": None}
        if self.use_gru_x3 and H == 128:
            pl = self._split_weights_t({"c": Fc, "vp": Fp, "vn": Fn, "hc": self.p("enc.gru_c_wh"),
                                        "hvp": self.p("enc.gru_vp_wh"), "hvn": self.p("enc.gru_vn_wh")})
            wt = {c: {"wi": pl[k], "wh": pl[hk][0]}
                  for c, k, hk in (("gru_c", "c", "hc"), ("gru_vp", "vp", "hvp"), ("gru_vn", "vn", "hvn"))}
            if self.use_gru_h2:
                h2, self._h2bad = self._split_weights_h2({
                    "gru_c": (Fc, self.p("enc.gru_c_wh")), "gru_vp": (Fp, self.p("enc.gru_vp_wh")),
                    "gru_vn": (Fn, self.p("enc.gru_vn_wh"))})
                for c in wt:
                    wt[c]["h2"] = h2[c]
        Hp, Hn, Hc = self._embed(b)
        tape: List[StepTape] = []
        ln = self.p("enc.ln")
        for l in range(self.L):
            GIN = e(Nc, 2 * H)  # [A+^T H_v+ | A-^T H_v-]
            _chk(L_.msat_clause_gather2(Hp.data_ptr(), Hn.data_ptr(), H, b.slots.data_ptr(), GIN.data_ptr(), 2 * H,
                                        Nc, H, 0, 0, self.stream), "clause_gather2")
            Hc1 = e(Nc, H)
            G4c = e(Nc, 4 * H) if save else None
            self._gru("gru_c", [(GIN.data_ptr(), 2 * H, 2 * H), (b.cdeg.data_ptr(), 4, 4)], Hc, ln[3 * l], Hc1, G4c,
                      Nc, wi=Fc, wt=wt["gru_c"])
            NV = e(Nv, 2 * H)  # [A+ H_c | A- H_c]
            _chk(L_.msat_var_gather2(Hc1.data_ptr(), Hc1.data_ptr(), H, b.ptr.data_ptr(), b.inc.data_ptr(),
                                     NV.data_ptr(), pp(NV, H), 2 * H, Nv, H, 0, self.stream), "var_gather2")
            outs = []
            for half, cell, Hx, k, F in ((0, "gru_vp", Hp, 3 * l + 1, Fp), (1, "gru_vn", Hn, 3 * l + 2, Fn)):
                Hx1 = e(Nv, H)
                G4 = e(Nv, 4 * H) if save else None
                # input [n_v | x | svf | n+ n- 0 0] against F rows [fold | Wi x/svf | count rows]
                self._gru(cell, [(pp(NV, half * H), 2 * H, H), (b.vfeat.data_ptr(), 8, 8)], Hx, ln[k], Hx1, G4, Nv,
                          wi=F, wt=wt[cell])
                outs.append((G4, Hx1))
            if save:
                tape.append(StepTape(Hp, Hn, Hc, GIN, G4c, NV, outs[0][0], outs[1][0]))
            Hp, Hn, Hc = outs[0][1], outs[1][1], Hc1
        return Hp, Hn, Hc, tape

    def _encode_backward_fused(self, b: GraphBatch, tape: List[StepTape], Hc_final, dHp, dHn, dHc):
        H, dev = self.H, self.device
        Nv, Nc = b.Nv, b.Nc
        e = lambda *shape: torch.empty(shape, dtype=torch.float32, device=dev)
        pp = self._ptr
        W3 = 3 * H
        ln, dln = self.p("enc.ln"), self.g("enc.ln")
        (Fc, Fp, Fn), (gFc, gFp, gFn) = self._fold_views()
        self._gF.zero_()
        # packed backward rows [dan | dar | daz | dan r] (4H): dGh = cols H..4H, dGi = cols 0..3H in gate
        # order (n, r, z); needs the x3 path (its F planes are split with the gate blocks rotated)
        packed = self.use_x3
        rot = 2 * H if packed else 0
        mats = {"wh_c": (self.p("enc.gru_c_wh"), 0), "wh_vp": (self.p("enc.gru_vp_wh"), 0),
                "wh_vn": (self.p("enc.gru_vn_wh"), 0), "Fc": (Fc[:2 * H], rot), "Fp": (Fp[:H], rot),
                "Fn": (Fn[:H], rot)}
        pl = self._split_weights(mats) if self.use_x3 else {k: None for k in mats}
        flags = 3 | (4 if packed else 0)
        dh2 = packed and self.use_dgrad_h2
        pl2, wbad = self._split_weights_f16(mats) if dh2 else (None, None)
        hx = lambda key, rexp: (pl2[key], wbad[key], rexp) if dh2 else None

        def dG_buffers(R):
            """-> (dGi ptr, dGh ptr, ld, keep-alive tensor)"""
            if packed:
                D = e(R, 4 * H)
                return D.data_ptr(), pp(D, H), 4 * H, D
            dGI, dGH = e(R, W3), e(R, W3)
            return dGI.data_ptr(), dGH.data_ptr(), W3, (dGI, dGH)

        h2 = packed and self.use_wgrad_h2
        need_rexp = h2 or dh2
        dual = h2 and dh2 and self.use_dual
        planes = dual and self.use_planes  # the packed rows as fp16x2 planes (read only by the dual products)
        if planes:
            flags |= 8

        def dF_wgrad(A, lda, dgi, ld, W, R, K, rexp):
            """W (dF rows, ld 3H) += A^T dGi; in packed rows dGi's gate blocks are (n | r z)."""
            if h2:
                self._wgrad_h2(A, lda, dgi, ld, rexp, W, W3, R, K, W3, rot=2 * H)
            elif packed:
                self._wgrad(A, lda, dgi, ld, W, W3, R, K, W3, rot=2 * H)
            else:
                self._wgrad(A, lda, dgi, ld, W, W3, R, K, W3)

        def Wh_wgrad(A, dgh, ld, W, R, rexp):
            """W (ld 3H) += A^T dGh (A = the cell's previous state, ld H)."""
            if h2:
                self._wgrad_h2(A, H, dgh, ld, rexp, W, W3, R, H, W3)
            else:
                self._wgrad(A, H, dgh, ld, W, W3, R, H, W3)

        def bwd(dHx, G4, Hx, ln_row, dgi, dgh, ldd, dHx0, dln_row, cell, feat, ldf, nfeat, dfeat, part, R, rexp):
            args = (dHx.data_ptr(), H, G4.data_ptr(), 4 * H, Hx.data_ptr(), H, ln_row, dgi, ldd, dgh, ldd,
                    dHx0.data_ptr(), H, dln_row, dln_row + 4 * H, self.g(f"enc.{cell}_bi").data_ptr(),
                    pp(self.g(f"enc.{cell}_bh"), 2 * H), feat, ldf, nfeat, dfeat, part.data_ptr(), R, H, flags)
            if need_rexp:
                _chk(L_.msat_gru_ln_bwd_g4fe(*args, rexp.data_ptr(), self.stream), "gru_ln_bwd_g4fe")
            else:
                _chk(L_.msat_gru_ln_bwd_g4f(*args, self.stream), "gru_ln_bwd_g4f")

        pp_addr = lambda ptr, col: ptr + 4 * col
        for l in range(self.L - 1, -1, -1):
            t = tape[l]
            dNV = e(Nv, 2 * H)
            dprev = {}
            for half, cell, Hx, G4, dHx, k, F, gF in ((0, "gru_vp", t.Hp, t.G4p, dHp, 3 * l + 1, Fp, gFp),
                                                     (1, "gru_vn", t.Hn, t.G4n, dHn, 3 * l + 2, Fn, gFn)):
                dgi, dgh, ldd, keep = dG_buffers(Nv)
                dHx0 = e(Nv, H)  # written (not accumulated) by the backward kernel: flags bit 1
                part = self.scr.get_part(int(L_.msat_gru_ln_bwd_partial_floats(Nv, H)))
                rexp = torch.empty(Nv, dtype=torch.int32, device=dev) if need_rexp else None
                # dF rows H..H+5 (x, svf, n+, n-) from the same pass: feature-weighted gate sums
                bwd(dHx, G4, Hx, pp(ln[k]), dgi, dgh, ldd, dHx0, pp(dln[k]), cell, b.vfeat.data_ptr(), 8, 6,
                    pp(gF[H]), part, Nv, rexp)
                wh, gwh = self.p(f"enc.{cell}_wh"), self.g(f"enc.{cell}_wh")
                sfx = cell[-2:]
                fk = "Fp" if half == 0 else "Fn"
                if dual:  # dh and d(gathered) in one launch, dWh and dF in another (same packed rows)
                    pb = dgi if planes else None
                    self._dgrad_dual((dgh, ldd, pl2["wh_" + sfx], pl["wh_" + sfx], wbad["wh_" + sfx], dHx0.data_ptr(),
                                      H, H, 1),
                                     (dgi, ldd, pl2[fk], pl[fk], wbad[fk], pp(dNV, half * H), 2 * H, H, 0), rexp, Nv, W3,
                                     pbase=pb)
                    self._wgrad_h2_dual((Hx.data_ptr(), H, dgh, ldd, gwh.data_ptr(), W3, H, W3, 0),
                                        (pp(t.NV, half * H), 2 * H, dgi, ldd, gF.data_ptr(), W3, H, W3, 2 * H), rexp, Nv,
                                        pbase=pb)
                else:
                    self._dgrad(dgh, ldd, wh, pl["wh_" + sfx], dHx0.data_ptr(), H, Nv, H, W3, 1, hx("wh_" + sfx, rexp))
                    Wh_wgrad(Hx.data_ptr(), dgh, ldd, gwh.data_ptr(), Nv, rexp)
                    # input path: d(gathered) and dF rows [fold | x/svf | counts]
                    self._dgrad(dgi, ldd, F, pl[fk], pp(dNV, half * H), 2 * H, Nv, H, W3, 0, hx(fk, rexp))
                    dF_wgrad(pp(t.NV, half * H), 2 * H, dgi, ldd, gF.data_ptr(), Nv, H, rexp)
                dprev[half] = dHx0
            # var gather backward: dH_c (+)= A+^T dNV+ + A-^T dNV-  (one merged clause gather)
            _chk(L_.msat_clause_gather2(dNV.data_ptr(), pp(dNV, H), 2 * H, b.slots.data_ptr(), dHc.data_ptr(), H, Nc,
                                        H, 1, 1, self.stream), "clause_gather2")
            # clause GRU
            dgi, dgh, ldd, keep = dG_buffers(Nc)
            dHc0 = e(Nc, H)
            part = self.scr.get_part(int(L_.msat_gru_ln_bwd_partial_floats(Nc, H)))
            rexp = torch.empty(Nc, dtype=torch.int32, device=dev) if need_rexp else None
            bwd(dHc, t.G4c, t.Hc, pp(ln[3 * l]), dgi, dgh, ldd, dHc0, pp(dln[3 * l]), "gru_c", b.cdeg.data_ptr(), 4, 2,
                pp(gFc[2 * H]), part, Nc, rexp)
            dGIN = e(Nc, 2 * H)
            if dual:
                pb = dgi if planes else None
                self._dgrad_dual((dgh, ldd, pl2["wh_c"], pl["wh_c"], wbad["wh_c"], dHc0.data_ptr(), H, H, 1),
                                 (dgi, ldd, pl2["Fc"], pl["Fc"], wbad["Fc"], dGIN.data_ptr(), 2 * H, 2 * H, 0), rexp, Nc,
                                 W3, pbase=pb)
                self._wgrad_h2_dual((t.Hc.data_ptr(), H, dgh, ldd, self.g("enc.gru_c_wh").data_ptr(), W3, H, W3, 0),
                                    (t.GIN.data_ptr(), 2 * H, dgi, ldd, gFc.data_ptr(), W3, 2 * H, W3, 2 * H), rexp, Nc,
                                    pbase=pb)
            else:
                self._dgrad(dgh, ldd, self.p("enc.gru_c_wh"), pl["wh_c"], dHc0.data_ptr(), H, Nc, H, W3, 1,
                            hx("wh_c", rexp))
                Wh_wgrad(t.Hc.data_ptr(), dgh, ldd, self.g("enc.gru_c_wh").data_ptr(), Nc, rexp)
                self._dgrad(dgi, ldd, Fc, pl["Fc"], dGIN.data_ptr(), 2 * H, Nc, 2 * H, W3, 0, hx("Fc", rexp))
                dF_wgrad(t.GIN.data_ptr(), 2 * H, dgi, ldd, gFc.data_ptr(), Nc, 2 * H, rexp)
            # clause gather backward: dH_v+/- (+)= A+/- dGIN+/-
            _chk(L_.msat_var_gather2(dGIN.data_ptr(), pp(dGIN, H), 2 * H, b.ptr.data_ptr(), b.inc.data_ptr(),
                                     dprev[0].data_ptr(), dprev[1].data_ptr(), H, Nv, H, 1, self.stream),
                 "var_gather2")
            dHp, dHn, dHc = dprev[0], dprev[1], dHc0
        self._embed_backward(b, dHp, dHn, dHc)
        self._unfuse_grads()

    def _encode_ref(self, b: GraphBatch, save: bool):
        H, dev = self.H, self.device
        Nv, Nc = b.Nv, b.Nc
        e = lambda *shape: torch.empty(shape, dtype=torch.float32, device=dev)
        pp = self._ptr
        Hp, Hn, Hc = self._embed(b)
        tape: List[StepTape] = []
        ln = self.p("enc.ln")
        for l in range(self.L):
            MV = e(Nv, 2 * H)
            self._gemm(Hp.data_ptr(), H, self.p("enc.phi_cp_w").data_ptr(), H, 0, MV.data_ptr(), 2 * H,
                       self.p("enc.phi_cp_b").data_ptr(), Nv, H, H)
            self._gemm(Hn.data_ptr(), H, self.p("enc.phi_cn_w").data_ptr(), H, 0, pp(MV, H), 2 * H,
                       self.p("enc.phi_cn_b").data_ptr(), Nv, H, H)
            GIN = e(Nc, 2 * H)
            _chk(L_.msat_clause_gather(MV.data_ptr(), 2 * H, b.slots.data_ptr(), GIN.data_ptr(), 2 * H, Nc, H, 0,
                                       self.stream), "clause_gather")
            Hc1 = e(Nc, H)
            G4c = e(Nc, 4 * H) if save else None
            self._gru("gru_c", [(GIN.data_ptr(), 2 * H, 2 * H)], Hc, ln[3 * l], Hc1, G4c, Nc)
            TPN = e(Nc, 2 * H)
            self._gemm(Hc1.data_ptr(), H, self.p("enc.phi_v_w").data_ptr(), 2 * H, 0, TPN.data_ptr(), 2 * H,
                       self.p("enc.phi_v_b").data_ptr(), Nc, 2 * H, H)
            NV = e(Nv, 2 * H)
            _chk(L_.msat_var_gather(TPN.data_ptr(), 2 * H, b.ptr.data_ptr(), b.inc.data_ptr(), NV.data_ptr(), 2 * H,
                                    Nv, H, 0, self.stream), "var_gather")
            outs = []
            for half, cell, Hx, k in ((0, "gru_vp", Hp, 3 * l + 1), (1, "gru_vn", Hn, 3 * l + 2)):
                # input [n_v | x | svf] (learner:75,78)
                Hx1 = e(Nv, H)
                G4 = e(Nv, 4 * H) if save else None
                self._gru(cell, [(pp(NV, half * H), 2 * H, H), (b.vfeat.data_ptr(), 8, 4)], Hx, ln[k], Hx1, G4, Nv)
                outs.append((G4, Hx1))
            if save:
                tape.append(StepTape(Hp, Hn, Hc, GIN, G4c, NV, outs[0][0], outs[1][0]))
            Hp, Hn, Hc = outs[0][1], outs[1][1], Hc1
        return Hp, Hn, Hc, tape

    def _encode_backward_ref(self, b: GraphBatch, tape: List[StepTape], Hc_final, dHp, dHn, dHc):
        H, dev = self.H, self.device
        Nv, Nc = b.Nv, b.Nc
        e = lambda *shape: torch.empty(shape, dtype=torch.float32, device=dev)
        pp = self._ptr
        ln, dln = self.p("enc.ln"), self.g("enc.ln")
        for l in range(self.L - 1, -1, -1):
            t = tape[l]
            Hc1 = tape[l + 1].Hc if l + 1 < self.L else Hc_final
            dNV = e(Nv, 2 * H)
            dprev = {}
            for half, cell, Hx, G4, dHx, k in ((0, "gru_vp", t.Hp, t.G4p, dHp, 3 * l + 1),
                                              (1, "gru_vn", t.Hn, t.G4n, dHn, 3 * l + 2)):
                dGI, dGH = e(Nv, 3 * H), e(Nv, 3 * H)
                dHx0 = torch.zeros((Nv, H), dtype=torch.float32, device=dev)
                part = self.scr.get_part(int(L_.msat_gru_ln_bwd_partial_floats(Nv, H)))
                _chk(L_.msat_gru_ln_bwd_g4(dHx.data_ptr(), H, G4.data_ptr(), 4 * H, Hx.data_ptr(), H, pp(ln[k]),
                                           dGI.data_ptr(), 3 * H, dGH.data_ptr(), 3 * H, dHx0.data_ptr(), H,
                                           pp(dln[k]), pp(dln[k], H), self.g(f"enc.{cell}_bi").data_ptr(),
                                           pp(self.g(f"enc.{cell}_bh"), 2 * H), part.data_ptr(), Nv, H, 1,
                                           self.stream), "gru_ln_bwd_g4")
                wi, wh = self.p(f"enc.{cell}_wi"), self.p(f"enc.{cell}_wh")
                gwi, gwh = self.g(f"enc.{cell}_wi"), self.g(f"enc.{cell}_wh")
                # hidden path
                self._gemm(dGH.data_ptr(), 3 * H, wh.data_ptr(), 3 * H, 1, dHx0.data_ptr(), H, None, Nv, H, 3 * H, 1)
                self._wgrad(Hx.data_ptr(), H, dGH.data_ptr(), 3 * H, gwh.data_ptr(), 3 * H, Nv, H, 3 * H)
                # input path [n_v | x | svf]
                self._gemm(dGI.data_ptr(), 3 * H, wi.data_ptr(), 3 * H, 1, pp(dNV, half * H), 2 * H, None, Nv, H,
                           3 * H, 0)
                self._wgrad(pp(t.NV, half * H), 2 * H, dGI.data_ptr(), 3 * H, gwi.data_ptr(), 3 * H, Nv, H, 3 * H)
                self._wgrad(b.vfeat.data_ptr(), 8, dGI.data_ptr(), 3 * H, pp(gwi[H]), 3 * H, Nv, 4, 3 * H)
                dprev[half] = dHx0
            # var gather backward = clause gather of dNV
            dTPN = e(Nc, 2 * H)
            _chk(L_.msat_clause_gather(dNV.data_ptr(), 2 * H, b.slots.data_ptr(), dTPN.data_ptr(), 2 * H, Nc, H, 0,
                                       self.stream), "clause_gather")
            self._gemm(dTPN.data_ptr(), 2 * H, self.p("enc.phi_v_w").data_ptr(), 2 * H, 1, dHc.data_ptr(), H, None,
                       Nc, H, 2 * H, 1)
            self._wgrad(Hc1.data_ptr(), H, dTPN.data_ptr(), 2 * H, self.g("enc.phi_v_w").data_ptr(), 2 * H, Nc, H,
                        2 * H)
            self._colsum(dTPN.data_ptr(), 2 * H, Nc, 2 * H, self.g("enc.phi_v_b").data_ptr())
            # clause GRU
            dGI, dGH = e(Nc, 3 * H), e(Nc, 3 * H)
            dHc0 = torch.zeros((Nc, H), dtype=torch.float32, device=dev)
            part = self.scr.get_part(int(L_.msat_gru_ln_bwd_partial_floats(Nc, H)))
            _chk(L_.msat_gru_ln_bwd_g4(dHc.data_ptr(), H, t.G4c.data_ptr(), 4 * H, t.Hc.data_ptr(), H, pp(ln[3 * l]),
                                       dGI.data_ptr(), 3 * H, dGH.data_ptr(), 3 * H, dHc0.data_ptr(), H,
                                       pp(dln[3 * l]), pp(dln[3 * l], H), self.g("enc.gru_c_bi").data_ptr(),
                                       pp(self.g("enc.gru_c_bh"), 2 * H), part.data_ptr(), Nc, H, 1, self.stream),
                 "gru_ln_bwd_g4")
            self._gemm(dGH.data_ptr(), 3 * H, self.p("enc.gru_c_wh").data_ptr(), 3 * H, 1, dHc0.data_ptr(), H, None,
                       Nc, H, 3 * H, 1)
            self._wgrad(t.Hc.data_ptr(), H, dGH.data_ptr(), 3 * H, self.g("enc.gru_c_wh").data_ptr(), 3 * H, Nc, H,
                        3 * H)
            dGIN = e(Nc, 2 * H)
            self._gemm(dGI.data_ptr(), 3 * H, self.p("enc.gru_c_wi").data_ptr(), 3 * H, 1, dGIN.data_ptr(), 2 * H,
                       None, Nc, 2 * H, 3 * H, 0)
            self._wgrad(t.GIN.data_ptr(), 2 * H, dGI.data_ptr(), 3 * H, self.g("enc.gru_c_wi").data_ptr(), 3 * H, Nc,
                        2 * H, 3 * H)
            # clause gather backward = var gather of dGIN
            dMV = e(Nv, 2 * H)
            _chk(L_.msat_var_gather(dGIN.data_ptr(), 2 * H, b.ptr.data_ptr(), b.inc.data_ptr(), dMV.data_ptr(),
                                    2 * H, Nv, H, 0, self.stream), "var_gather")
            for half, nm, Hx, dst in ((0, "phi_cp", t.Hp, dprev[0]), (1, "phi_cn", t.Hn, dprev[1])):
                self._gemm(pp(dMV, half * H), 2 * H, self.p(f"enc.{nm}_w").data_ptr(), H, 1, dst.data_ptr(), H,
                           None, Nv, H, H, 1)
                self._wgrad(Hx.data_ptr(), H, pp(dMV, half * H), 2 * H, self.g(f"enc.{nm}_w").data_ptr(), H, Nv, H, H)
                self._colsum(pp(dMV, half * H), 2 * H, Nv, H, self.g(f"enc.{nm}_b").data_ptr())
            dHp, dHn, dHc = dprev[0], dprev[1], dHc0
        self._embed_backward(b, dHp, dHn, dHc)

    # ------------------------------------------------------------ heads ----
    def _gr(self, b: GraphBatch):
        return b.vbase.data_ptr(), b.nv.data_ptr(), b.cbase.data_ptr(), b.nc.data_ptr()

    def critic_head(self, b: GraphBatch, Hp, Hn, Hc, ht: HeadTape):
        H, S = self.H, b.S
        pooled = torch.empty((S, 6 * H), device=self.device)
        _chk(L_.msat_critic_pool(Hp.data_ptr(), Hn.data_ptr(), Hc.data_ptr(), H, *self._gr(b), b.G, S,
                                 pooled.data_ptr(), self.stream), "critic_pool")
        c0 = torch.empty((S, 128), device=self.device)
        self._gemm(pooled.data_ptr(), 6 * H, self.p("crit.d0_w").data_ptr(), 128, 0, c0.data_ptr(), 128,
                   self.p("crit.d0_b").data_ptr(), S, 128, 6 * H)
        _chk(L_.msat_relu(c0.data_ptr(), c0.numel(), self.stream), "relu")
        c1 = torch.empty((S, 64), device=self.device)
        self._gemm(c0.data_ptr(), 128, self.p("crit.d1_w").data_ptr(), 64, 0, c1.data_ptr(), 64,
                   self.p("crit.d1_b").data_ptr(), S, 64, 128)
        _chk(L_.msat_relu(c1.data_ptr(), c1.numel(), self.stream), "relu")
        val = torch.empty((S,), device=self.device)
        self._gemm(c1.data_ptr(), 64, self.p("crit.out_w").data_ptr(), 1, 0, val.data_ptr(), 1,
                   self.p("crit.out_b").data_ptr(), S, 1, 64)
        ht.pooled, ht.c0, ht.c1 = pooled, c0, c1
        return val

    def critic_head_backward(self, b, Hp, Hn, Hc, ht: HeadTape, dval, dHp, dHn, dHc):
        H, S, dev = self.H, b.S, self.device
        dc1 = torch.empty((S, 64), device=dev)
        self._gemm(dval.data_ptr(), 1, self.p("crit.out_w").data_ptr(), 1, 1, dc1.data_ptr(), 64, None, S, 64, 1)
        self._wgrad(ht.c1.data_ptr(), 64, dval.data_ptr(), 1, self.g("crit.out_w").data_ptr(), 1, S, 64, 1)
        self._colsum(dval.data_ptr(), 1, S, 1, self.g("crit.out_b").data_ptr())
        _chk(L_.msat_relu_bwd(dc1.data_ptr(), ht.c1.data_ptr(), dc1.numel(), self.stream), "relu_bwd")
        dc0 = torch.empty((S, 128), device=dev)
        self._gemm(dc1.data_ptr(), 64, self.p("crit.d1_w").data_ptr(), 64, 1, dc0.data_ptr(), 128, None, S, 128, 64)
        self._wgrad(ht.c0.data_ptr(), 128, dc1.data_ptr(), 64, self.g("crit.d1_w").data_ptr(), 64, S, 128, 64)
        self._colsum(dc1.data_ptr(), 64, S, 64, self.g("crit.d1_b").data_ptr())
        _chk(L_.msat_relu_bwd(dc0.data_ptr(), ht.c0.data_ptr(), dc0.numel(), self.stream), "relu_bwd")
        dpooled = torch.empty((S, 6 * H), device=dev)
        self._gemm(dc0.data_ptr(), 128, self.p("crit.d0_w").data_ptr(), 128, 1, dpooled.data_ptr(), 6 * H, None, S,
                   6 * H, 128)
        self._wgrad(ht.pooled.data_ptr(), 6 * H, dc0.data_ptr(), 128, self.g("crit.d0_w").data_ptr(), 128, S, 6 * H,
                    128)
        self._colsum(dc0.data_ptr(), 128, S, 128, self.g("crit.d0_b").data_ptr())
        _chk(L_.msat_critic_pool_bwd(Hp.data_ptr(), Hn.data_ptr(), Hc.data_ptr(), H, *self._gr(b), b.G, S,
                                     dpooled.data_ptr(), dHp.data_ptr(), dHn.data_ptr(), dHc.data_ptr(), self.stream),
             "critic_pool_bwd")

    def actor_head(self, b: GraphBatch, Hp, Hn, Hc, ht: HeadTape):
        H, S, A, M, CW, dev = self.H, b.S, self.A, self.M, self.CW, self.device
        SA = S * A
        my = torch.empty((SA * M, 2 * H), device=dev)
        ctx = torch.empty((SA, CW), device=dev)
        _chk(L_.msat_actor_pool(Hp.data_ptr(), Hn.data_ptr(), Hc.data_ptr(), H, *self._gr(b), b.G, S, A, M, self.base,
                                self.rem, self.p("actor.id_emb").data_ptr(), self.E, my.data_ptr(), ctx.data_ptr(),
                                self.stream), "actor_pool")
        ht.my, ht.ctx = my, ctx
        pp = self._ptr
        if self.mode == 0:
            w1 = self.p("actor.flip_d_w")
            Pm = torch.empty((SA, 128), device=dev)
            self._gemm(ctx.data_ptr(), CW, pp(w1[2 * H]), 128, 0, Pm.data_ptr(), 128, None, SA, 128, CW)
            h1 = torch.empty((SA * M, 128), device=dev)
            self._gemm(my.data_ptr(), 2 * H, w1.data_ptr(), 128, 0, h1.data_ptr(), 128,
                       self.p("actor.flip_d_b").data_ptr(), SA * M, 128, 2 * H)
            _chk(L_.msat_bcast_add_relu(h1.data_ptr(), Pm.data_ptr(), SA, M, 128, self.stream), "bcast_add_relu")
            fl = torch.empty((SA * M,), device=dev)
            self._gemm(h1.data_ptr(), 128, self.p("actor.flip_o_w").data_ptr(), 1, 0, fl.data_ptr(), 1,
                       self.p("actor.flip_o_b").data_ptr(), SA * M, 1, 128)
            n1 = torch.empty((SA, 64), device=dev)
            self._gemm(ctx.data_ptr(), CW, self.p("actor.noop_d_w").data_ptr(), 64, 0, n1.data_ptr(), 64,
                       self.p("actor.noop_d_b").data_ptr(), SA, 64, CW)
            _chk(L_.msat_relu(n1.data_ptr(), n1.numel(), self.stream), "relu")
            no = torch.empty((SA,), device=dev)
            self._gemm(n1.data_ptr(), 64, self.p("actor.noop_o_w").data_ptr(), 1, 0, no.data_ptr(), 1,
                       self.p("actor.noop_o_b").data_ptr(), SA, 1, 64)
            logits = torch.empty((S, A, M + 1), device=dev)
            _chk(L_.msat_assemble_logits(fl.data_ptr(), no.data_ptr(), SA, A, M, self.base, self.rem,
                                         logits.data_ptr(), self.stream), "assemble_logits")
            ht.h1, ht.n1 = h1, n1
            return logits
        w0 = self.p("actor.d0_w")
        Pm = torch.empty((SA, 128), device=dev)
        self._gemm(pp(ctx, 5 * H), CW, pp(w0[2 * H]), 128, 0, Pm.data_ptr(), 128, None, SA, 128, self.E)
        h1 = torch.empty((SA * M, 128), device=dev)
        self._gemm(my.data_ptr(), 2 * H, w0.data_ptr(), 128, 0, h1.data_ptr(), 128, self.p("actor.d0_b").data_ptr(),
                   SA * M, 128, 2 * H)
        _chk(L_.msat_bcast_add_relu(h1.data_ptr(), Pm.data_ptr(), SA, M, 128, self.stream), "bcast_add_relu")
        h2 = torch.empty((SA * M, 64), device=dev)
        self._gemm(h1.data_ptr(), 128, self.p("actor.d1_w").data_ptr(), 64, 0, h2.data_ptr(), 64,
                   self.p("actor.d1_b").data_ptr(), SA * M, 64, 128)
        _chk(L_.msat_relu(h2.data_ptr(), h2.numel(), self.stream), "relu")
        logits = torch.empty((S, A, M, 2), device=dev)
        self._gemm(h2.data_ptr(), 64, self.p("actor.out_w").data_ptr(), 2, 0, logits.data_ptr(), 2,
                   self.p("actor.out_b").data_ptr(), SA * M, 2, 64)
        _chk(L_.msat_mask_var_logits(logits.data_ptr(), SA, A, M, self.base, self.rem, self.stream), "mask_logits")
        ht.h1, ht.h2 = h1, h2
        return logits

    def actor_head_backward(self, b, ht: HeadTape, dlogits, dHp, dHn, dHc):
        H, S, A, M, CW, dev = self.H, b.S, self.A, self.M, self.CW, self.device
        SA = S * A
        pp = self._ptr
        dmy = torch.empty((SA * M, 2 * H), device=dev)
        dctx = torch.empty((SA, CW), device=dev)
        if self.mode == 0:
            dfl = torch.empty((SA * M,), device=dev)
            dno = torch.empty((SA,), device=dev)
            _chk(L_.msat_split_dlogits(dlogits.data_ptr(), SA, M, dfl.data_ptr(), dno.data_ptr(), self.stream),
                 "split_dlogits")
            dh1 = torch.empty((SA * M, 128), device=dev)
            self._gemm(dfl.data_ptr(), 1, self.p("actor.flip_o_w").data_ptr(), 1, 1, dh1.data_ptr(), 128, None,
                       SA * M, 128, 1)
            self._wgrad(ht.h1.data_ptr(), 128, dfl.data_ptr(), 1, self.g("actor.flip_o_w").data_ptr(), 1, SA * M, 128, 1)
            self._colsum(dfl.data_ptr(), 1, SA * M, 1, self.g("actor.flip_o_b").data_ptr())
            _chk(L_.msat_relu_bwd(dh1.data_ptr(), ht.h1.data_ptr(), dh1.numel(), self.stream), "relu_bwd")
            dP = torch.empty((SA, 128), device=dev)
            _chk(L_.msat_group_sum(dh1.data_ptr(), SA, M, 128, dP.data_ptr(), self.stream), "group_sum")
            w1, gw1 = self.p("actor.flip_d_w"), self.g("actor.flip_d_w")
            self._gemm(dh1.data_ptr(), 128, w1.data_ptr(), 128, 1, dmy.data_ptr(), 2 * H, None, SA * M, 2 * H, 128)
            self._wgrad(ht.my.data_ptr(), 2 * H, dh1.data_ptr(), 128, gw1.data_ptr(), 128, SA * M, 2 * H, 128)
            self._colsum(dh1.data_ptr(), 128, SA * M, 128, self.g("actor.flip_d_b").data_ptr())
            self._gemm(dP.data_ptr(), 128, pp(w1[2 * H]), 128, 1, dctx.data_ptr(), CW, None, SA, CW, 128)
            self._wgrad(ht.ctx.data_ptr(), CW, dP.data_ptr(), 128, pp(gw1[2 * H]), 128, SA, CW, 128)
            dn1 = torch.empty((SA, 64), device=dev)
            self._gemm(dno.data_ptr(), 1, self.p("actor.noop_o_w").data_ptr(), 1, 1, dn1.data_ptr(), 64, None, SA, 64, 1)
            self._wgrad(ht.n1.data_ptr(), 64, dno.data_ptr(), 1, self.g("actor.noop_o_w").data_ptr(), 1, SA, 64, 1)
            self._colsum(dno.data_ptr(), 1, SA, 1, self.g("actor.noop_o_b").data_ptr())
            _chk(L_.msat_relu_bwd(dn1.data_ptr(), ht.n1.data_ptr(), dn1.numel(), self.stream), "relu_bwd")
            self._gemm(dn1.data_ptr(), 64, self.p("actor.noop_d_w").data_ptr(), 64, 1, dctx.data_ptr(), CW, None, SA,
                       CW, 64, 1)
            self._wgrad(ht.ctx.data_ptr(), CW, dn1.data_ptr(), 64, self.g("actor.noop_d_w").data_ptr(), 64, SA, CW, 64)
            self._colsum(dn1.data_ptr(), 64, SA, 64, self.g("actor.noop_d_b").data_ptr())
        else:
            dh2 = torch.empty((SA * M, 64), device=dev)
            self._gemm(dlogits.data_ptr(), 2, self.p("actor.out_w").data_ptr(), 2, 1, dh2.data_ptr(), 64, None, SA * M,
                       64, 2)
            self._wgrad(ht.h2.data_ptr(), 64, dlogits.data_ptr(), 2, self.g("actor.out_w").data_ptr(), 2, SA * M, 64, 2)
            self._colsum(dlogits.data_ptr(), 2, SA * M, 2, self.g("actor.out_b").data_ptr())
            _chk(L_.msat_relu_bwd(dh2.data_ptr(), ht.h2.data_ptr(), dh2.numel(), self.stream), "relu_bwd")
            dh1 = torch.empty((SA * M, 128), device=dev)
            self._gemm(dh2.data_ptr(), 64, self.p("actor.d1_w").data_ptr(), 64, 1, dh1.data_ptr(), 128, None, SA * M,
                       128, 64)
            self._wgrad(ht.h1.data_ptr(), 128, dh2.data_ptr(), 64, self.g("actor.d1_w").data_ptr(), 64, SA * M, 128, 64)
            self._colsum(dh2.data_ptr(), 64, SA * M, 64, self.g("actor.d1_b").data_ptr())
            _chk(L_.msat_relu_bwd(dh1.data_ptr(), ht.h1.data_ptr(), dh1.numel(), self.stream), "relu_bwd")
            dP = torch.empty((SA, 128), device=dev)
            _chk(L_.msat_group_sum(dh1.data_ptr(), SA, M, 128, dP.data_ptr(), self.stream), "group_sum")
            w0, gw0 = self.p("actor.d0_w"), self.g("actor.d0_w")
            self._gemm(dh1.data_ptr(), 128, w0.data_ptr(), 128, 1, dmy.data_ptr(), 2 * H, None, SA * M, 2 * H, 128)
            self._wgrad(ht.my.data_ptr(), 2 * H, dh1.data_ptr(), 128, gw0.data_ptr(), 128, SA * M, 2 * H, 128)
            self._colsum(dh1.data_ptr(), 128, SA * M, 128, self.g("actor.d0_b").data_ptr())
            dctx.zero_()
            self._gemm(dP.data_ptr(), 128, pp(w0[2 * H]), 128, 1, pp(dctx, 5 * H), CW, None, SA, self.E, 128)
            self._wgrad(pp(ht.ctx, 5 * H), CW, dP.data_ptr(), 128, pp(gw0[2 * H]), 128, SA, self.E, 128)
        did = torch.empty((SA, self.E), device=dev)
        _chk(L_.msat_actor_pool_bwd(H, *self._gr(b), b.G, S, A, M, self.base, self.rem, self.E, dmy.data_ptr(),
                                    dctx.data_ptr(), dHp.data_ptr(), dHn.data_ptr(), dHc.data_ptr(), did.data_ptr(),
                                    self.stream), "actor_pool_bwd")
        self._colsum(did.data_ptr(), A * self.E, S, A * self.E, self.g("actor.id_emb").data_ptr())

    # ---------------------------------------------------------- top level ----
    def forward(self, b: GraphBatch, actor: bool = True, critic: bool = True, save: bool = False):
        Hp, Hn, Hc, tape = self.encode(b, save)
        ht = HeadTape()
        logits = self.actor_head(b, Hp, Hn, Hc, ht) if actor else None
        value = self.critic_head(b, Hp, Hn, Hc, ht) if critic else None
        state = (Hp, Hn, Hc, tape, ht) if save else None
        return logits, value, state

    def backward(self, b: GraphBatch, state, dlogits: Optional[torch.Tensor], dvalue: Optional[torch.Tensor]):
        """Accumulate parameter gradients (self.grads += ...) for upstream grads of logits / value."""
        Hp, Hn, Hc, tape, ht = state
        dHp = torch.zeros_like(Hp)
        dHn = torch.zeros_like(Hn)
        dHc = torch.zeros_like(Hc)
        if dvalue is not None:
            self.critic_head_backward(b, Hp, Hn, Hc, ht, dvalue, dHp, dHn, dHc)
        if dlogits is not None:
            self.actor_head_backward(b, ht, dlogits, dHp, dHn, dHc)
        self.encode_backward(b, tape, Hc, dHp, dHn, dHc)

    def adam_step(self, lr: float, grad_scale: float = 1.0, b1=0.9, b2=0.999, eps=1e-8,
                  first_bad: Optional[torch.Tensor] = None):
        """One optax.adam step.  first_bad (device int32 scalar, INT32_MAX when clean): set to the smallest
        Adam count whose update left a parameter non-finite (msat_adam_checked; no host sync)."""
        self.adam_count += 1
        _chk(L_.msat_adam_checked(self.params.data_ptr(), self.grads.data_ptr(), self.adam_m.data_ptr(),
                                  self.adam_v.data_ptr(), self.size, float(lr), b1, b2, eps, self.adam_count,
                                  float(grad_scale), first_bad.data_ptr() if first_bad is not None else None,
                                  self.stream), "adam")


def path_switches(precision: str) -> dict:
    """GNNActorCritic's kernel-path switches for one MARLSAT_PRECISION value (README "Kernel-path switches"):
    'fp16x2' = phi folded, fp16x2 GRU forward and data / weight gradients (bf16x3 fixups); 'bf16x3' = phi
    folded, the bf16x3 kernels throughout; 'fp32' = fp32 MFMA kernels in the reference's operation order
    (phi not folded)."""
    if precision not in PRECISION_CODES:
        raise ValueError(f"precision must be one of {sorted(PRECISION_CODES)}, got {precision!r}")
    split, h2 = precision != "fp32", precision == "fp16x2"
    return {"fuse_phi": split, "use_x3": split, "use_gru_x3": split, "use_gru_h2": h2, "use_dgrad_h2": h2,
            "use_wgrad_h2": h2}


def set_precision(precision: str) -> dict:
    """Switch the process's matrix arithmetic (the class switches above and the library's weight-gradient path,
    msat_set_precision) to one precision path; returns the previous switches (restore_precision undoes it)."""
    prev = {k: getattr(GNNActorCritic, k) for k in path_switches(precision)}
    prev["_code"] = int(L_.msat_get_precision())
    for k, v in path_switches(precision).items():
        setattr(GNNActorCritic, k, v)
    _lib.check(L_.msat_set_precision(PRECISION_CODES[precision]), "msat_set_precision")
    return prev


def restore_precision(prev: dict) -> None:
    for k, v in prev.items():
        if k != "_code":
            setattr(GNNActorCritic, k, v)
    _lib.check(L_.msat_set_precision(prev["_code"]), "msat_set_precision")
