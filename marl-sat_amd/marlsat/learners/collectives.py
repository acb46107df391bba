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

``dist`` is torch.distributed (its "nccl" backend is RCCL on ROCm) or a ``CapiComm``: the same calls
over the library's own RCCL communicator (``msat_comm_init`` / ``msat_allreduce_sum``,
include/marlsat_net.h), the route a host without torch takes through the C-ABI
(``MARLSAT_COLLECTIVES=capi`` in bench.py).
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


class CapiComm:
    """torch.distributed-shaped handle (``is_initialized``, ``get_world_size``, ``get_rank``,
    ``all_reduce``: the calls this module makes) over one RCCL communicator of libmarlsat.so.  Tensors
    must be contiguous fp32 / fp64 device tensors; the SUM runs in place on the current stream."""

    def __init__(self, rank: int, world: int, uid: bytes):
        import ctypes

        from .. import _lib

        self._lib, self.rank, self.world = _lib, int(rank), int(world)
        n = int(_lib.lib.msat_comm_id_bytes())
        if len(uid) != n:
            raise ValueError(f"communicator id must be {n} bytes, got {len(uid)}")
        buf = (ctypes.c_uint8 * n).from_buffer_copy(uid)
        handle = ctypes.c_void_p()
        _lib.check(_lib.lib.msat_comm_init(buf, self.rank, self.world, ctypes.byref(handle)), "msat_comm_init")
        self._comm = handle

    @staticmethod
    def unique_id() -> bytes:
        import ctypes

        from .. import _lib

        n = int(_lib.lib.msat_comm_id_bytes())
        buf = (ctypes.c_uint8 * n)()
        _lib.check(_lib.lib.msat_comm_unique_id(buf), "msat_comm_unique_id")
        return bytes(buf)

    @classmethod
    def from_dist(cls, dist) -> "CapiComm":
        """Rank 0 draws the id and broadcasts it over an initialised torch.distributed group."""
        rank, world = dist.get_rank(), dist.get_world_size()
        box = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        return cls(rank, world, box[0])

    def is_initialized(self) -> bool:
        return self._comm is not None

    def get_world_size(self) -> int:
        return self.world

    def get_rank(self) -> int:
        return self.rank

    def all_reduce(self, t: torch.Tensor, op=None) -> None:
        if op is not None and "SUM" not in str(op).upper():
            raise ValueError("CapiComm.all_reduce supports SUM only")
        if not (t.is_cuda and t.is_contiguous() and t.dtype in (torch.float32, torch.float64)):
            raise ValueError("CapiComm.all_reduce needs a contiguous fp32 / fp64 device tensor")
        self._lib.check(self._lib.lib.msat_allreduce_sum(self._comm, t.data_ptr(), t.numel(),
                                                         1 if t.dtype == torch.float64 else 0,
                                                         self._lib.stream_ptr(t.device)), "msat_allreduce_sum")

    def destroy(self) -> None:
        if self._comm is not None:
            self._lib.check(self._lib.lib.msat_comm_destroy(self._comm), "msat_comm_destroy")
            self._comm = None


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
