"""Host mirror of the device reset RNG (Philox4x32-10) — test infrastructure.

Bit-exact restatement of ``philox4x32_10`` / ``reset_rng_block`` in
``marl-sat_amd/csrc/common.h``; lets tests replay an RNG-driven device reset
with explicit problem indices / assignments through the oracle.
"""
import numpy as np

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
_MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 over uint32 arrays (broadcasting)."""
    c0, c1, c2, c3 = (np.asarray(x, dtype=np.uint32) for x in (c0, c1, c2, c3))
    k0 = np.asarray(k0, dtype=np.uint32)
    k1 = np.asarray(k1, dtype=np.uint32)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = _M0 * c0.astype(np.uint64)
            p1 = _M1 * c2.astype(np.uint64)
            hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & _MASK).astype(np.uint32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & _MASK).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
            k0 = (k0 + _W0).astype(np.uint32)
            k1 = (k1 + _W1).astype(np.uint32)
    return c0, c1, c2, c3


def reset_draws(seed: int, counter: int, num_envs: int, num_vars: int, num_problems: int):
    """(problem_idx (B,), assignment (B,V) uint8) the device RNG draws for a reset call."""
    k0, k1 = np.uint32(seed & 0xFFFFFFFF), np.uint32((seed >> 32) & 0xFFFFFFFF)
    c0, c1 = np.uint32(counter & 0xFFFFFFFF), np.uint32((counter >> 32) & 0xFFFFFFFF)
    envs = np.arange(num_envs, dtype=np.uint32)
    r0 = philox4x32_10(c0, c1, envs, np.uint32(0), k0, k1)[0]
    pidx = ((r0.astype(np.uint64) * np.uint64(num_problems)) >> np.uint64(32)).astype(np.int32)
    nblk = (num_vars + 127) // 128
    words = np.stack(
        philox4x32_10(c0, c1, envs[:, None], np.arange(1, nblk + 1, dtype=np.uint32)[None, :], k0, k1), axis=-1
    )  # (B, nblk, 4)
    v = np.arange(num_vars)
    w = words[:, v >> 7, (v >> 5) & 3]
    x = ((w >> (v & 31).astype(np.uint32)) & 1).astype(np.uint8)
    return pidx, x
