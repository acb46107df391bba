"""Device ops of the MAPPO loop that sit outside the network (thin wrappers over the C-ABI)."""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from .. import _lib


class GaeWorkspace:
    def __init__(self, T: int, B: int, device):
        n = int(_lib.lib.msat_gae_workspace_bytes(T, B))
        self.buf = torch.empty((n + 7) // 8, dtype=torch.float64, device=device)
        self.T, self.B = T, B


def gae(reward: torch.Tensor, value: torch.Tensor, done: torch.Tensor, last_val: torch.Tensor, gamma: float,
        gae_lambda: float, *, normalize: bool = True, out: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
        workspace: Optional[GaeWorkspace] = None):
    """GAE + global advantage normalisation (learner:504-532) on the device.

    reward: (T,B) team reward, or (T,B,A) per-agent reward of which agent 0 is used
    (``reward[..., 0]``, learner:514).  done (T,B) bool/uint8, value (T,B), last_val (B,).
    Returns (advantages, targets); advantages are normalised when ``normalize``.
    """
    T, B = value.shape
    if reward.dim() == 3:
        stride = reward.shape[2]
    else:
        stride = 1
    for t, n in ((reward, "reward"), (value, "value"), (last_val, "last_val")):
        _lib.require_device(t, n)
        if t.dtype != torch.float32:
            raise TypeError(f"{n} must be float32")
    d = done.to(torch.uint8).contiguous()
    if tuple(d.shape) != (T, B) or tuple(last_val.shape) != (B,) or tuple(reward.shape[:2]) != (T, B):
        raise ValueError("gae: shapes must be reward (T,B[,A]), value/done (T,B), last_val (B,)")
    adv, tgt = out if out is not None else (torch.empty_like(value), torch.empty_like(value))
    ws = workspace if workspace is not None else GaeWorkspace(T, B, value.device)
    _lib.check(
        _lib.lib.msat_gae(T, B, reward.data_ptr(), stride, d.data_ptr(), value.data_ptr(), last_val.data_ptr(),
                          float(gamma), float(gamma * gae_lambda), 1 if normalize else 0, adv.data_ptr(),
                          tgt.data_ptr(), ws.buf.data_ptr(), _lib.stream_ptr(value.device)),
        "msat_gae",
    )
    return adv, tgt
