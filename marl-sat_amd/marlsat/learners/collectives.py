"""The learner's cross-rank exchanges, in one place.

One process per GPU, each with its own env shard, problem-pool stream and a full
replica of the parameters and Adam state.  The ranks meet only at:

  * ``allreduce_grads`` -- once per PPO minibatch, a SUM all-reduce of the flat fp32
    gradient buffer (one RCCL call over xGMI, ~2.8 MB at the reference's H=128, L=16);
    Adam then applies ``grad_scale = 1/world``.  Every rank's loss is a mean over its
    own minibatch slice of equal size, so the rank mean equals the gradient of the
    union minibatch (learner:597-650: losses are means over MB / MB*A / entropy rows);
  * ``global_moments`` -- once per cycle, (sum, sum of squares, count) of the raw GAE
    advantages in fp64, so the normalisation is global over all T*B*world samples as
    in the reference (learner:530-532, population std + 1e-8);
  * ``allreduce_sums`` -- once per cycle, the metric sums (learner:661-719).

With ``dist is None`` or world 1 every function is the identity, so the
single-GPU learner pays nothing.  The functions take torch tensors on any device:
the CPU ``gloo`` tests (tests/test_dist_cpu.py) run exactly this code.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch


def world_size(dist) -> int:
    return dist.get_world_size() if dist is not None and dist.is_initialized() else 1


def allreduce_grads(grads: torch.Tensor, dist) -> float:
    """In-place SUM over ranks of the flat gradient buffer; returns the Adam grad_scale (1/world)."""
    w = world_size(dist)
    if w > 1:
        dist.all_reduce(grads)
    return 1.0 / w


def allreduce_sums(t: torch.Tensor, dist) -> torch.Tensor:
    if world_size(dist) > 1:
        dist.all_reduce(t)
    return t


def global_moments(local_sums: torch.Tensor, n_local: int, dist) -> Tuple[float, float]:
    """(mean, std + 1e-8) of the union of every rank's advantages from local fp64 [sum, sum_sq]."""
    mom = torch.cat([local_sums.to(torch.float64).reshape(2),
                     torch.tensor([float(n_local)], dtype=torch.float64, device=local_sums.device)])
    allreduce_sums(mom, dist)
    s1, s2, cnt = mom.tolist()
    mean = s1 / cnt
    return mean, math.sqrt(max(s2 / cnt - mean * mean, 0.0)) + 1e-8


def init_from_env(backend: Optional[str] = None):
    """torchrun-style init (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT); returns the dist module or None."""
    import os

    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return None
    import torch.distributed as dist

    if not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group(backend, **kw)
    return dist
