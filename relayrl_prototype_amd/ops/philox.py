"""Host oracle of the device Philox4x32-10 counter RNG (csrc/kernels/common.h).

Vectorised over numpy uint32 arrays so tests can reproduce every draw the rollout /
sampling kernels make (same key, same counter -> same bits).
"""
from __future__ import annotations

import numpy as np

_M0 = np.uint64(0xD2511F53)
_M1 = np.uint64(0xCD9E8D57)
_W0 = np.uint32(0x9E3779B9)
_W1 = np.uint32(0xBB67AE85)


def philox4x32(c0, c1, c2, c3, k0, k1, rounds: int = 10):
    c0, c1, c2, c3 = (np.asarray(x, dtype=np.uint32).copy() for x in (c0, c1, c2, c3))
    k0 = np.asarray(k0, dtype=np.uint32).copy()
    k1 = np.asarray(k1, dtype=np.uint32).copy()
    with np.errstate(over="ignore"):
        for _ in range(rounds):
            p0 = _M0 * c0.astype(np.uint64)
            p1 = _M1 * c2.astype(np.uint64)
            lo0 = (p0 & np.uint64(0xFFFFFFFF)).astype(np.uint32)
            hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
            lo1 = (p1 & np.uint64(0xFFFFFFFF)).astype(np.uint32)
            hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
            k0 = (k0 + _W0).astype(np.uint32)
            k1 = (k1 + _W1).astype(np.uint32)
    return c0, c1, c2, c3


def u01(x) -> np.ndarray:
    """Same mapping as the device: top 24 bits -> [0, 1)."""
    return (np.asarray(x, dtype=np.uint32) >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def uniforms(seed: int, step: int, rows, tag: int = 0):
    """The 4 uniforms the kernels draw for stream ``rows`` at global step ``step``."""
    rows = np.asarray(rows, dtype=np.uint64)
    c0 = (rows & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    n = c0.shape
    c1 = np.full(n, step & 0xFFFFFFFF, dtype=np.uint32)
    c2 = np.full(n, (step >> 32) & 0xFFFFFFFF, dtype=np.uint32)
    c3 = np.full(n, tag, dtype=np.uint32)
    k0 = np.full(n, seed & 0xFFFFFFFF, dtype=np.uint32)
    k1 = np.full(n, (seed >> 32) & 0xFFFFFFFF, dtype=np.uint32)
    r = philox4x32(c0, c1, c2, c3, k0, k1)
    return tuple(u01(x) for x in r)
