"""Closed-form deterministic input generators shared by the golden-vector
script, the parity tests and the CPU baseline.

Test infrastructure only.  Every value is a pure function of (shape, seed):
a splitmix64 hash of the flat element index, so the same arrays come out on
any host, numpy version or GPU box without shipping the inputs themselves.
"""
from __future__ import annotations

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _splitmix64(idx: np.ndarray, seed: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = idx.astype(np.uint64) + np.uint64(seed) * _GOLDEN + _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def synth_uniform(shape, seed: int) -> np.ndarray:
    """U[0,1) float32 with 24-bit resolution (exactly representable)."""
    n = int(np.prod(shape))
    z = _splitmix64(np.arange(n, dtype=np.uint64), seed)
    u = (z >> np.uint64(40)).astype(np.float64) * (1.0 / (1 << 24))
    return u.astype(np.float32).reshape(shape)


def synth_normal(shape, seed: int, start: int = 0) -> np.ndarray:
    """N(0,1) float32 by Box-Muller on two independent hash streams.  start:
    flat index of the first element, so a big array can be made in slices
    (synth_normal(s, seed, k * n) == synth_normal((K, *s), seed)[k])."""
    n = int(np.prod(shape))
    idx = np.arange(start, start + n, dtype=np.uint64)
    z1 = _splitmix64(idx, seed)
    z2 = _splitmix64(idx, seed + 7919)
    u1 = ((z1 >> np.uint64(11)).astype(np.float64) + 1.0) * (1.0 / (1 << 53))
    u2 = (z2 >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))
    r = np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)
    return r.astype(np.float32).reshape(shape)


def synth_timesteps(n: int, T: int, seed: int) -> np.ndarray:
    z = _splitmix64(np.arange(n, dtype=np.uint64), seed)
    return (z % np.uint64(T)).astype(np.int64)
