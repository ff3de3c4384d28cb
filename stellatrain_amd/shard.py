"""Bucket sharding across GPUs of one node.

The reference compresses every gradient bucket as an independent task
(engine/core.cpp:1052-1087); the only cross-call state is the per-key AIMD
threshold (thresholdv16.cpp:84-97).  So the multi-GPU path partitions buckets,
not data: each rank owns a fixed set of keys (key-affine placement, so a key's
threshold stays resident on its owner), compresses them with no collective on
the data path, and the job's throughput is all ranks' bytes over the slowest
rank's time.  The only collectives are the timing barrier and the max-reduce of
the elapsed time (bench.py), and the optional result gather in tests.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .engine import owner_of

__all__ = ["ShardPlan", "c4_sizes"]


def c4_sizes(count: int = 1024, lo: int = 65536, hi: int = 16777216, seed: int = 4) -> list[int]:
    """Config 4's bucket stream: n log-uniform in [lo, hi] floats (256 KiB ..
    64 MiB), seeded, rounded to whole 16-float lines."""
    rng = np.random.default_rng(seed)
    n = np.exp(rng.uniform(np.log(lo), np.log(hi), size=count))
    return [int(x) // 16 * 16 for x in n]


@dataclass
class ShardPlan:
    """Placement of a bucket list over `world` ranks."""

    sizes: list[int]
    world: int

    def __post_init__(self):
        self.owner = owner_of(self.sizes, self.world)

    def local(self, rank: int) -> list[int]:
        """Bucket ids owned by `rank`, in bucket order."""
        return [i for i, o in enumerate(self.owner) if o == rank]

    def key(self, bucket: int) -> str:
        """Persistent key of a bucket ("layer@param", task.cpp:56-61)."""
        return f"{bucket}@grad"

    def local_bytes(self, rank: int) -> int:
        return 4 * sum(self.sizes[i] for i in self.local(rank))

    def imbalance(self) -> float:
        """max / mean of per-rank bytes (1.0 = perfect)."""
        b = [self.local_bytes(r) for r in range(self.world)]
        return max(b) / (sum(b) / self.world) if sum(b) else 1.0
