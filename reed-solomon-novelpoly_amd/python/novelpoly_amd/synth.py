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


def decode_rows(present: np.ndarray, n: int, k: int, fast_nq: tuple = (1, 2, 4)) -> int:
    """Shard rows the fused-locator reconstruct kernel reads for one payload: it
    decodes from the shortest prefix of q*k rows (q in ``fast_nq``, q*k <= n)
    that holds k present rows (kernels_fast.hip, rec_tile), reading only the
    present rows of that prefix.  Used for the algorithmic byte count."""
    present = np.asarray(present).astype(bool)
    for q in fast_nq:
        if q * k <= n and int(present[: q * k].sum()) >= k:
            return int(present[: q * k].sum())
    return int(present[:n].sum())
