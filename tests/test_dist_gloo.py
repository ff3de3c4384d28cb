"""Multi-rank bucket sharding on CPU (world size 2, gloo).

The N>1 path of bench.py shards buckets over ranks by key (stellatrain_amd.
shard.ShardPlan) with no collective on the data path; each key's AIMD state
lives on its owner.  Here each rank runs the codec restatement (the oracle,
standing in for the device on a CPU-only box) over its own buckets for a few
iterations; rank 0 gathers the per-bucket digests and checks them against a
single-process run: every bucket exactly once, identical outputs and threshold
trajectories for any world size, and the max-over-ranks time reduction the
bench uses.
"""
from __future__ import annotations

import hashlib
import json
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SIZES = [1000, 65536, 100013, 4096 + 7, 33, 250000, 17, 131072, 70000, 9999]
ITERS = 3
RATIO = 0.99


def _digests(bucket_ids, sizes):
    sys.path.insert(0, ROOT)
    from oracle.oracle import Oracle
    from stellatrain_amd.engine import merge_numel
    from stellatrain_amd.shard import ShardPlan
    from stellatrain_amd.synth import seed_for, synth
    o = Oracle()
    h = o.tv16_new()
    plan = ShardPlan(sizes, 1)
    out = {}
    for b in bucket_ids:
        key = plan.key(b)
        n = sizes[b]
        k = merge_numel(n, RATIO)
        hs = hashlib.sha256()
        traj = []
        for it in range(ITERS):
            cnt, idx, val = o.tv16_compress(h, key, synth(n, seed_for(b, it)), k)
            hs.update(np.int64(cnt).tobytes() + idx[:cnt].tobytes() + val[:cnt].tobytes())
            t, inc = o.tv16_state(h, key)
            traj.append(int(np.float32(t).view(np.uint32)))
        out[b] = (hs.hexdigest(), traj)
    o.tv16_free(h)
    return out


def _worker(rank, world, port, result_path):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    from stellatrain_amd.shard import ShardPlan
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    plan = ShardPlan(SIZES, world)
    mine = plan.local(rank)
    dig = _digests(mine, SIZES)
    gathered = [None] * world
    dist.all_gather_object(gathered, {"rank": rank, "buckets": mine, "digests": dig})
    el = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)  # bench.py's max-over-ranks time
    if rank == 0:
        with open(result_path, "w") as f:
            json.dump({"gathered": gathered, "max_time": float(el.item())}, f)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_plan_covers_every_bucket_once():
    sys.path.insert(0, ROOT)
    from stellatrain_amd.shard import ShardPlan, c4_sizes
    sizes = c4_sizes()
    assert len(sizes) == 1024 and min(sizes) >= 65536 - 16 and max(sizes) <= 16777216
    for world in (1, 2, 4, 8):
        p = ShardPlan(sizes, world)
        got = sorted(i for r in range(world) for i in p.local(r))
        assert got == list(range(len(sizes)))
        assert p.imbalance() < 1.005  # longest-first greedy over 1024 buckets


def test_gloo_world2_matches_single_process(tmp_path):
    torch = pytest.importorskip("torch")
    import torch.multiprocessing as mp
    world = 2
    path = str(tmp_path / "res.json")
    mp.start_processes(_worker, args=(world, _free_port(), path), nprocs=world, join=True, start_method="spawn")
    res = json.load(open(path))
    assert res["max_time"] == float(world)
    seen = {}
    for g in res["gathered"]:
        for b in g["buckets"]:
            assert b not in seen, "bucket owned by two ranks"
            seen[b] = g["digests"][str(b)]
    assert sorted(seen) == list(range(len(SIZES)))
    single = _digests(range(len(SIZES)), SIZES)
    for b in range(len(SIZES)):
        assert tuple(seen[b][0:1]) == (single[b][0],), f"bucket {b} output differs across world sizes"
        assert seen[b][1] == single[b][1], f"bucket {b} threshold trajectory differs"
