"""marlsat — MI355X-native marl-sat hot path (batched SAT env + MAPPO rollout math).

Host side in Python over a thin ctypes C-ABI (``include/marlsat.h``) into
hand-written HIP kernels for gfx950 (``marl-sat_amd/csrc``).  PyTorch-ROCm
tensors are the device array container; there is no CPU fallback.
"""
from . import _lib  # noqa: F401  (fails loudly when libmarlsat.so is missing)
from .envs.multi_agent_sat_env import ObsDict, ProblemPool, SATEnv, SATState  # noqa: F401

__all__ = ["SATEnv", "SATState", "ProblemPool", "ObsDict"]
