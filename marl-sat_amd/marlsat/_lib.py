"""ctypes binding of libmarlsat.so (the C-ABI declared in include/marlsat.h).

The product path has no CPU fallback: if the shared library is missing or
cannot be loaded this module raises ImportError, and every op raises
RuntimeError with the library's error message when a call fails.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_float, c_int32, c_size_t, c_uint64, c_void_p

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MARLSAT_LIB", os.path.join(_HERE, "lib", "libmarlsat.so"))

OBS_I32, OBS_I8 = 0, 1
MAX_GROUPS = 8  # MSAT_MAX_GROUPS
REWARD_SPARSE, REWARD_PBRS, REWARD_SINGLE_DELTA = 0, 1, 2


class EnvDesc(ctypes.Structure):
    _fields_ = [
        ("num_envs", c_int32),
        ("num_vars", c_int32),
        ("num_clauses", c_int32),
        ("clause_width", c_int32),
        ("num_agents", c_int32),
        ("max_vars_per_agent", c_int32),
        ("max_steps", c_int32),
        ("action_mode", c_int32),
        ("reward_mode", c_int32),
        ("obs_dtype", c_int32),
        ("num_problems", c_int32),
        ("r_clause", c_float),
        ("r_sat", c_float),
        ("gamma", c_float),
    ]


class EnvStateC(ctypes.Structure):
    _fields_ = [
        ("assign", c_void_p),
        ("clause_sat", c_void_p),
        ("clause_ntrue", c_void_p),
        ("num_unsat", c_void_p),
        ("step", c_void_p),
        ("done", c_void_p),
        ("problem_idx", c_void_p),
        ("reset_queue", c_void_p),  # nullable: timed-out resets in workgroups of their own (include/marlsat.h)
        ("reset_serial", ctypes.c_uint32),
    ]


class PoolC(ctypes.Structure):
    _fields_ = [("lits", c_void_p), ("rel", c_void_p), ("nbr", c_void_p)]


class StepOutC(ctypes.Structure):
    _fields_ = [
        ("reward", c_void_p),
        ("done", c_void_p),
        ("solved", c_void_p),
        ("num_unsat", c_void_p),
        ("episode_step", c_void_p),
        ("clock_stamps", c_void_p),  # diagnostics (bench.py's clock), NULL otherwise
    ]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"marlsat: native library not found at {LIB_PATH}; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)"
        )
    lib = ctypes.CDLL(LIB_PATH)
    P = c_void_p
    sig = {
        "msat_last_error": (ctypes.c_char_p, []),
        "msat_version": (c_int32, []),
        "msat_pool_pack": (c_int32, [P, c_int32, c_int32, c_int32, c_int32, P, P, P]),
        "msat_pool_agent_tables": (c_int32, [POINTER(EnvDesc), P, P, P, P]),
        "msat_env_reset": (
            c_int32, [POINTER(EnvDesc), POINTER(PoolC), POINTER(EnvStateC), P, P, P, c_uint64, c_uint64, P, P]
        ),
        "msat_env_step": (
            c_int32,
            [POINTER(EnvDesc), POINTER(PoolC), POINTER(EnvStateC), P, c_int32, P, P, c_uint64, c_uint64,
             POINTER(StepOutC), P, P],
        ),
        "msat_env_reset_grouped": (
            c_int32, [c_int32, POINTER(EnvDesc), POINTER(PoolC), POINTER(EnvStateC), c_uint64, c_uint64, P, P]
        ),
        "msat_env_step_grouped": (
            c_int32, [c_int32, POINTER(EnvDesc), POINTER(PoolC), POINTER(EnvStateC), P, c_int32, c_uint64, c_uint64,
                      POINTER(StepOutC), P, P]
        ),
        "msat_env_obs": (c_int32, [POINTER(EnvDesc), POINTER(PoolC), POINTER(EnvStateC), P, P]),
        "msat_env_masks": (c_int32, [POINTER(EnvDesc), POINTER(PoolC), POINTER(EnvStateC), P, P, P, P]),
        "msat_clause_features": (c_int32, [POINTER(EnvDesc), POINTER(EnvStateC), P, P]),
        "msat_clause_sat_features": (c_int32, [POINTER(EnvDesc), POINTER(EnvStateC), P, P]),
        "msat_bc_greedy_labels": (c_int32, [POINTER(EnvDesc), P, P, P, c_float, P, P, P]),
        "msat_static_var_features": (c_int32, [P, c_int32, c_int32, c_int32, P, P]),
        "msat_reset_queue_words": (c_size_t, [c_int32]),
        "msat_gae_workspace_bytes": (c_size_t, [c_int32, c_int32]),
        "msat_gae": (
            c_int32,
            [c_int32, c_int32, P, c_int32, P, P, P, c_float, c_float, c_int32, P, P, P, P],
        ),
    }
    # marlsat_net.h
    sig["msat_gemm"] = (c_int32, [P, c_int32, P, c_int32, c_int32, P, c_int32, P, c_int32, c_int32, c_int32, c_int32,
                                  P])
    sig["msat_gemm_wgrad_workspace_bytes"] = (c_size_t, [c_int32, c_int32, c_int32])
    sig["msat_gemm_wgrad"] = (c_int32, [P, c_int32, P, c_int32, P, c_int32, c_int32, c_int32, c_int32, c_int32, P, P])
    sig["msat_gemm_wgrad_h2"] = (c_int32, [P, c_int32, P, c_int32, P, P, c_int32, c_int32, c_int32, c_int32, c_int32,
                                           c_int32, P, P])
    sig["msat_gemm_wgrad_rot"] = (c_int32, [P, c_int32, P, c_int32, P, c_int32, c_int32, c_int32, c_int32, c_int32,
                                            c_int32, P, P])
    I, F, Z, U = c_int32, c_float, c_size_t, c_uint64
    sig["msat_assemble_graph_batch"] = (I, [I, I, I, I, I] + [P] * 26 + [I, I, P])
    sig["msat_clause_gather"] = (I, [P, I, P, P, I, I, I, I, P])
    sig["msat_var_gather"] = (I, [P, I, P, P, P, I, I, I, I, P])
    sig["msat_split_bf16x3"] = (I, [P, I, I, I, P, P])
    sig["msat_split_bf16x3_rot"] = (I, [P, I, I, I, I, P, P])
    sig["msat_gemm_x3"] = (I, [P, I, P, P, I, P, I, I, I, I, P])
    sig["msat_split_f16x2_rot"] = (I, [P, I, I, I, I, P, P, P])
    sig["msat_gemm_h2"] = (I, [P, I, P, P, P, P, P, I, P, I, I, I, I, P])
    sig["msat_permutation"] = (I, [I, U, U, P, P])
    sig["msat_gather_rows"] = (I, [P, I, I, P, P, P, P])
    sig["msat_cycle_metrics"] = (I, [I, P, P, P, P, P, P, P, P, P])
    sig["msat_graph_bases"] = (I, [I, P, P, P, P, P, P, P])
    sig["msat_gemm_h2_dual"] = (I, [P, I, P, P, P, P, I, I, I, P, I, P, P, P, P, I, I, I, P, I, I, P])
    sig["msat_gemm_wgrad_dual_workspace_bytes"] = (c_size_t, [I, I, I, I, I])
    sig["msat_gemm_wgrad_h2_dual"] = (I, [P, I, P, I, P, I, I, I, I, P, I, P, I, P, I, I, I, I, P, I, I, P, P])
    sig["msat_gemm_h2_dual_planes"] = (I, [P, I, P, P, P, P, I, I, I, P, I, P, P, P, P, I, I, I, I, P, I, I, P])
    sig["msat_gemm_wgrad_h2_dual_planes"] = (I, [P, I, P, I, P, I, I, I, I, P, I, P, I, P, I, I, I, I, I, P, I, I, P,
                                                  P])
    sig["msat_clause_gather2"] = (I, [P, P, I, P, P, I, I, I, I, I, P])
    sig["msat_var_gather2"] = (I, [P, P, I, P, P, P, P, I, I, I, I, P])
    sig["msat_gru_ln_fwd"] = (I, [P, I, P, I, P, I, P, P, P, I, I, I, P])
    sig["msat_gru_ln_fused_fwd"] = (I, [P, I, I, P, I, I, P, I, I, P, I, P, P, P, P, P, P, P, I, P, I, I, I, P])
    sig["msat_gru_ln_fused_fwd_x3r"] = (I, [P, I, I, P, I, I, P, I, I, P, I, P, I, P, P, P, P, P, P, I, P, I, I, I, P])
    sig["msat_split_bf16x3_t"] = (I, [P, I, I, I, I, P, P])
    sig["msat_gru_ln_fused_fwd_h2r"] = (I, [P, I, I, P, I, I, P, I, I, P, I, P, P, P, P, I, P, P, P, P, P, I, P, I, I, I,
                                             P, P, P])
    sig["msat_split_f16x2_t"] = (I, [P, I, I, I, I, P, P, P])
    sig["msat_gru_ln_bwd_g4"] = (I, [P, I, P, I, P, I, P, P, I, P, I, P, I, P, P, P, P, P, I, I, I, P])
    sig["msat_gru_ln_bwd_g4f"] = (I, [P, I, P, I, P, I, P, P, I, P, I, P, I, P, P, P, P, P, I, I, P, P, I, I, I, P])
    sig["msat_gru_ln_bwd_g4fe"] = (I, [P, I, P, I, P, I, P, P, I, P, I, P, I, P, P, P, P, P, I, I, P, P, I, I, I, P, P])
    sig["msat_gru_ln_bwd_partial_floats"] = (Z, [I, I])
    sig["msat_gru_ln_bwd"] = (I, [P, I, P, I, P, I, P, I, P, P, I, P, I, P, I, P, P, P, I, I, I, P])
    sig["msat_colsum_workspace_floats"] = (Z, [I, I])
    sig["msat_colsum"] = (I, [P, I, I, I, P, I, P, P])
    sig["msat_relu"] = (I, [P, Z, P])
    sig["msat_relu_bwd"] = (I, [P, P, Z, P])
    sig["msat_critic_pool"] = (I, [P, P, P, I, P, P, P, P, I, I, P, P])
    sig["msat_critic_pool_bwd"] = (I, [P, P, P, I, P, P, P, P, I, I, P, P, P, P, P])
    sig["msat_actor_pool"] = (I, [P, P, P, I, P, P, P, P, I, I, I, I, I, I, P, I, P, P, P])
    sig["msat_actor_pool_bwd"] = (I, [I, P, P, P, P, I, I, I, I, I, I, I, P, P, P, P, P, P, P])
    sig["msat_bcast_add_relu"] = (I, [P, P, I, I, I, P])
    sig["msat_group_sum"] = (I, [P, I, I, I, P, P])
    sig["msat_assemble_logits"] = (I, [P, P, I, I, I, I, I, P, P])
    sig["msat_mask_var_logits"] = (I, [P, I, I, I, I, I, P])
    sig["msat_split_dlogits"] = (I, [P, I, I, P, P, P])
    sig["msat_sample_actions"] = (I, [P, I, I, I, U, U, P, P, P])
    sig["msat_ppo_loss"] = (I, [P, I, I, I, I, I, I, P, P, P, P, P, P, F, F, F, F, I, P, P, P, P, P])
    sig["msat_gemm_f64acc"] = (I, [P, I, I, P, I, I, P, I, I, I, I, I, P])
    sig["msat_adam"] = (I, [P, P, P, P, Z, F, F, F, F, I, F, P])
    sig["msat_adam_checked"] = (I, [P, P, P, P, Z, F, F, F, F, I, F, P, P])
    sig["msat_set_precision"] = (I, [I])
    sig["msat_get_precision"] = (I, [])
    sig["msat_moments"] = (I, [P, Z, P, P, P])
    sig["msat_standardize"] = (I, [P, Z, F, F, P])
    sig["msat_comm_id_bytes"] = (Z, [])
    sig["msat_comm_unique_id"] = (I, [P])
    sig["msat_comm_init"] = (I, [P, I, I, P])
    sig["msat_allreduce_sum"] = (I, [P, P, Z, I, P])
    sig["msat_comm_destroy"] = (I, [P])
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()
ABI_VERSION = 3  # msat_version() of the header this binding follows (msat_env_state with the reset queue)
if lib.msat_version() != ABI_VERSION:
    raise ImportError(f"marlsat: {LIB_PATH} has C-ABI version {lib.msat_version()}, this binding needs {ABI_VERSION}; "
                      "rebuild it (make -C marl-sat_amd)")

_probe = None


def probe_lib():
    """libmarlsat_probe.so: diagnostic store / expansion probes (csrc/marlsat_probe.h) for profiles/*.py only."""
    global _probe
    if _probe is None:
        d = ctypes.CDLL(os.path.join(os.path.dirname(LIB_PATH), "libmarlsat_probe.so"))
        P = c_void_p
        for name, args in (("msat_probe_fill", [P, c_size_t, c_int32, c_int32, c_int32, P]),
                           ("msat_probe_fill_chunked", [P, c_size_t, c_int32, c_int32, c_int32, P]),
                           ("msat_probe_obs_expand", [P, c_int32, c_int32, c_int32, P, P, P, c_int32, P]),
                           ("msat_probe_fill_rows", [P, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32,
                                                     P]),
                           ("msat_probe_strip_read", [P, c_int32, c_int32, c_int32, c_int32, P, P]),
                           ("msat_probe_l2_read", [P, c_int32, c_int32, c_int32, c_int32, c_int32, P, P])):
            fn = getattr(d, name)
            fn.restype, fn.argtypes = c_int32, args
        _probe = d
    return _probe

# Every symbol include/marlsat*.h declares (checked by tests/test_capi.py).
EXPORTED = (
    "msat_comm_id_bytes",
    "msat_comm_unique_id",
    "msat_comm_init",
    "msat_allreduce_sum",
    "msat_comm_destroy",
    "msat_moments",
    "msat_standardize",
    "msat_assemble_graph_batch",
    "msat_clause_gather",
    "msat_var_gather",
    "msat_gru_ln_fused_fwd_x3r",
    "msat_split_bf16x3_t",
    "msat_gru_ln_fused_fwd_h2r",
    "msat_split_f16x2_t",
    "msat_split_bf16x3",
    "msat_split_bf16x3_rot",
    "msat_gemm_x3",
    "msat_split_f16x2_rot",
    "msat_gemm_h2",
    "msat_permutation",
    "msat_gather_rows",
    "msat_cycle_metrics",
    "msat_graph_bases",
    "msat_gemm_h2_dual",
    "msat_gemm_wgrad_dual_workspace_bytes",
    "msat_gemm_wgrad_h2_dual",
    "msat_gemm_h2_dual_planes",
    "msat_gemm_wgrad_h2_dual_planes",
    "msat_clause_gather2",
    "msat_var_gather2",
    "msat_gru_ln_fwd",
    "msat_gru_ln_fused_fwd",
    "msat_gru_ln_bwd_g4",
    "msat_gru_ln_bwd_g4f",
    "msat_gru_ln_bwd_g4fe",
    "msat_gru_ln_bwd_partial_floats",
    "msat_gru_ln_bwd",
    "msat_colsum_workspace_floats",
    "msat_colsum",
    "msat_relu",
    "msat_relu_bwd",
    "msat_critic_pool",
    "msat_critic_pool_bwd",
    "msat_actor_pool",
    "msat_actor_pool_bwd",
    "msat_bcast_add_relu",
    "msat_group_sum",
    "msat_assemble_logits",
    "msat_mask_var_logits",
    "msat_split_dlogits",
    "msat_sample_actions",
    "msat_ppo_loss",
    "msat_adam",
    "msat_adam_checked",
    "msat_set_precision",
    "msat_get_precision",
    "msat_gemm",
    "msat_gemm_f64acc",
    "msat_gemm_wgrad_workspace_bytes",
    "msat_gemm_wgrad",
    "msat_gemm_wgrad_rot",
    "msat_gemm_wgrad_h2",
    "msat_last_error",
    "msat_version",
    "msat_pool_pack",
    "msat_pool_agent_tables",
    "msat_env_reset",
    "msat_env_step",
    "msat_env_reset_grouped",
    "msat_clause_sat_features",
    "msat_bc_greedy_labels",
    "msat_env_step_grouped",
    "msat_env_obs",
    "msat_env_masks",
    "msat_clause_features",
    "msat_static_var_features",
    "msat_gae_workspace_bytes",
    "msat_gae",
    "msat_reset_queue_words",
)


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib.msat_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (code {rc}): {msg}")


def ptr(t) -> int | None:
    """Device pointer of a tensor (None for None)."""
    if t is None:
        return None
    return t.data_ptr()


def stamps_ptr(t, num_envs: int) -> int | None:
    """Device pointer of an optional msat_step_out.clock_stamps buffer: int64, contiguous, at least 8 words per
    env (include/marlsat.h: (B, 8)); the kernel writes all eight, so a smaller buffer is refused here."""
    if t is None:
        return None
    if t.dtype not in (torch.int64, torch.uint64) or not t.is_contiguous() or t.numel() < 8 * num_envs:
        raise ValueError(f"clock_stamps must be a contiguous int64 tensor of >= 8 * {num_envs} elements ((B, 8)), "
                         f"got {tuple(t.shape)} {t.dtype}")
    return t.data_ptr()


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_device(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(f"marlsat: {what} must be a device (cuda/hip) tensor; there is no CPU path")
    if not t.is_contiguous():
        raise RuntimeError(f"marlsat: {what} must be contiguous")
