"""Minimal jaxmarl-style spaces (``jaxmarl.environments.spaces``) used by SATEnv.

Only the attributes the reference reads are provided: ``n`` / ``num_categories``
/ ``shape`` / ``low`` / ``high`` / ``dtype`` and a device ``sample``.
"""
from __future__ import annotations

from typing import Sequence, Tuple

import torch


class Space:
    dtype = torch.int32


class Discrete(Space):
    def __init__(self, num_categories: int, dtype=torch.int32):
        self.n = self.num_categories = int(num_categories)
        self.shape: Tuple[int, ...] = ()
        self.dtype = dtype

    def sample(self, generator: torch.Generator, batch: Sequence[int] = (), device=None):
        return torch.randint(0, self.n, tuple(batch), generator=generator, dtype=self.dtype, device=device)

    def contains(self, x) -> bool:
        x = torch.as_tensor(x)
        return bool(((x >= 0) & (x < self.n)).all())


class MultiDiscrete(Space):
    def __init__(self, num_categories: Sequence[int], dtype=torch.int32):
        self.num_categories = list(int(n) for n in num_categories)
        self.shape = (len(self.num_categories),)
        self.dtype = dtype

    def sample(self, generator: torch.Generator, batch: Sequence[int] = (), device=None):
        hi = torch.tensor(self.num_categories, device=device)
        u = torch.rand(tuple(batch) + self.shape, generator=generator, device=device)
        return (u * hi).floor().to(self.dtype)

    def contains(self, x) -> bool:
        x = torch.as_tensor(x)
        hi = torch.tensor(self.num_categories, device=x.device)
        return bool(((x >= 0) & (x < hi)).all())


class Box(Space):
    def __init__(self, low, high, shape: Tuple[int, ...], dtype=torch.int32):
        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), dtype

    def contains(self, x) -> bool:
        x = torch.as_tensor(x)
        return tuple(x.shape[-len(self.shape):]) == self.shape and bool(((x >= self.low) & (x <= self.high)).all())
