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
REWARD_SPARSE, REWARD_PBRS = 0, 1


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
        "msat_env_obs": (c_int32, [POINTER(EnvDesc), POINTER(PoolC), POINTER(EnvStateC), P, P]),
        "msat_env_masks": (c_int32, [POINTER(EnvDesc), POINTER(PoolC), POINTER(EnvStateC), P, P, P, P]),
        "msat_clause_features": (c_int32, [POINTER(EnvDesc), POINTER(EnvStateC), P, P]),
        "msat_static_var_features": (c_int32, [P, c_int32, c_int32, c_int32, P, P]),
        "msat_gae_workspace_bytes": (c_size_t, [c_int32, c_int32]),
        "msat_gae": (
            c_int32,
            [c_int32, c_int32, P, c_int32, P, P, P, c_float, c_float, c_int32, P, P, P, P],
        ),
    }
    sig["msat_debug_fill"] = (c_int32, [P, c_size_t, c_int32, c_int32, c_int32, P])  # marlsat_debug.h
    sig["msat_debug_fill_chunked"] = (c_int32, [P, c_size_t, c_int32, c_int32, c_int32, P])
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()

# Every symbol include/marlsat.h declares (checked by tests/test_capi.py).
EXPORTED = (
    "msat_last_error",
    "msat_version",
    "msat_pool_pack",
    "msat_pool_agent_tables",
    "msat_env_reset",
    "msat_env_step",
    "msat_env_obs",
    "msat_env_masks",
    "msat_clause_features",
    "msat_static_var_features",
    "msat_gae_workspace_bytes",
    "msat_gae",
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


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_device(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(f"marlsat: {what} must be a device (cuda/hip) tensor; there is no CPU path")
    if not t.is_contiguous():
        raise RuntimeError(f"marlsat: {what} must be contiguous")
