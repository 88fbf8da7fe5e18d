"""Deterministic synthetic workloads.

* payload bytes: splitmix64 stream, seed 0x5EED_0000 + payload_index,
  little-endian u64 words;
* erasures: partial Fisher-Yates over [0, n) driven by splitmix64 with seed
  0xE7A5_0000 + payload_index.

The BASELINE configs (BASELINE.json ``configs``) are listed in CONFIGS with
the effective (n, k) that ``CodeParams::derive_parameters`` yields
(mod.rs:43-61).
"""
from __future__ import annotations

import numpy as np

GAMMA = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)

CONFIGS = {
    # id: CodeParams::derive_parameters(n_wanted, k_wanted) -> effective (n, k)
    1: dict(n_wanted=16, k_wanted=8, n=16, k=8, payload=4096, batch=1, erase=8),
    2: dict(n_wanted=256, k_wanted=86, n=256, k=64, payload=64 * 1024, batch=4096, erase=None),
    3: dict(n_wanted=1024, k_wanted=342, n=1024, k=256, payload=1 << 20, batch=1024, erase=342),
    4: dict(n_wanted=4096, k_wanted=1366, n=4096, k=1024, payload=4 << 20, batch=256, erase=2730),
    5: dict(n_wanted=1024, k_wanted=342, n=1024, k=256, payload=1 << 20, batch=8192, erase=342),
}


def _mix(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        return z ^ (z >> np.uint64(31))


def splitmix64_words(seed: int, count: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        idx = np.arange(1, count + 1, dtype=np.uint64)
        return _mix(np.uint64(seed) + idx * GAMMA)


def payload(index: int, nbytes: int) -> bytes:
    words = splitmix64_words(0x5EED0000 + index, (nbytes + 7) // 8)
    return words.astype("<u8").tobytes()[:nbytes]


def payload_array(index: int, nbytes: int) -> np.ndarray:
    return np.frombuffer(payload(index, nbytes), dtype=np.uint8)


class SplitMix64:
    def __init__(self, seed: int):
        self.state = seed & 0xFFFFFFFFFFFFFFFF

    def next(self) -> int:
        self.state = (self.state + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = self.state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        return z ^ (z >> 31)


def erasure_indices(index: int, n: int, count: int) -> np.ndarray:
    """Partial Fisher-Yates: the first `count` entries of a random permutation of [0,n)."""
    rng = SplitMix64(0xE7A50000 + index)
    perm = list(range(n))
    for i in range(count):
        j = i + rng.next() % (n - i)
        perm[i], perm[j] = perm[j], perm[i]
    return np.array(sorted(perm[:count]), dtype=np.int64)


def present_mask(index: int, n: int, count: int) -> np.ndarray:
    m = np.ones(n, dtype=np.uint8)
    m[erasure_indices(index, n, count)] = 0
    return m


def _s64(x: int) -> int:
    """A u64 constant as the int64 with the same bits (torch has no uint64 math)."""
    return x - (1 << 64) if x >= 1 << 63 else x


def payload_batch_dev(lo: int, hi: int, nbytes: int, device):
    """Payloads lo..hi-1 as a (hi - lo) x nbytes uint8 torch tensor on `device`,
    bit-identical to :func:`payload` (splitmix64 in int64 arithmetic: products
    wrap mod 2^64, logical shifts by masking).  Generates the bench's 1 GiB
    batches in milliseconds instead of seconds of host work."""
    import torch

    words = (nbytes + 7) // 8
    seeds = torch.arange(lo, hi, dtype=torch.int64, device=device) + 0x5EED0000
    idx = torch.arange(1, words + 1, dtype=torch.int64, device=device)
    out = torch.empty((hi - lo, words), dtype=torch.int64, device=device)
    gamma, m1, m2 = _s64(0x9E3779B97F4A7C15), _s64(0xBF58476D1CE4E5B9), _s64(0x94D049BB133111EB)

    def lsr(z, s):
        return (z >> s) & ((1 << (64 - s)) - 1)

    step = max(1, (1 << 24) // max(1, words))  # bound the temporaries to ~16M words
    for b0 in range(0, hi - lo, step):
        z = seeds[b0:b0 + step, None] + idx[None, :] * gamma
        z = (z ^ lsr(z, 30)) * m1
        z = (z ^ lsr(z, 27)) * m2
        out[b0:b0 + step] = z ^ lsr(z, 31)
    return out.view(torch.uint8)[:, :nbytes].contiguous() if nbytes % 8 else out.view(torch.uint8)
