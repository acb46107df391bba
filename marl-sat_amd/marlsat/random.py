"""Keys for the device RNG (stand-in for ``jax.random`` keys on this path).

A ``Key`` is (seed, counter): the device kernels draw Philox4x32-10 words keyed
by ``seed`` at counter ``(counter, env, word)``.  ``split`` derives
independent child keys deterministically, so a rollout reproduces from its
seed exactly as a JAX program reproduces from its PRNGKey (but with different
streams: JAX threefry is not reproducible here).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Union

_MIX = 0x9E3779B97F4A7C15
_MASK = (1 << 64) - 1


def _splitmix(x: int) -> int:
    x = (x + _MIX) & _MASK
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _MASK
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _MASK
    return x ^ (x >> 31)


@dataclass(frozen=True)
class Key:
    seed: int
    counter: int = 0

    def fold(self, n: int) -> "Key":
        return Key(self.seed, (self.counter + n) & _MASK)


def PRNGKey(seed: int) -> Key:
    return Key(_splitmix(int(seed) & _MASK), 0)


def split(key: Key, num: int = 2) -> List[Key]:
    base = _splitmix(key.seed ^ _splitmix(key.counter))
    return [Key(_splitmix(base + i + 1), 0) for i in range(num)]


def as_key(key: Union[None, int, Key]) -> Key:
    if key is None:
        return Key(0, 0)
    if isinstance(key, Key):
        return key
    return PRNGKey(int(key))
