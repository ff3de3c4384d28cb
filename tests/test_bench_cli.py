"""bench.py's multi-GPU entry on CPU: ``--gpus 2`` relaunches the script under
torch.distributed.run (one process per rank) before any device call; each
rank runs the headline step on its own keys (weak scaling) and then its
ShardPlan share of the C4 bucket stream (BASELINE.json configs[3], the ``c4``
sub-object, strong scaling) -- here with the CPU restatement standing in for
the device (``--backend oracle``, gloo, scaled-down sizes) -- and rank 0
prints the one JSON line with n_gpus equal to the ranks that joined.  N = 1
carries the same c4 sub-object, so the 1..N curve has one workload.
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(args, tmp_path):
    dump = tmp_path / "shards.json"
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--backend", "oracle", "--c4-count", "48",
                        "--c4-hi", "131072", "--c4-sweeps", "1", "--mib", "1", "--keys", "4", "--steps", "2",
                        "--warmup", "1", "--dump-shards", str(dump),
                        "--master-port", str(_free_port())] + args,
                       capture_output=True, text=True, timeout=600, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # only rank 0 prints
    return json.loads(lines[0]), json.load(open(dump))


def test_bench_gpus2_spawns_two_ranks_with_disjoint_shards(tmp_path):
    out, shards = _run(["--gpus", "2"], tmp_path)
    assert out["n_gpus"] == 2 and out["rccl_world_size"] == 2
    assert out["scaling"] == "weak" and out["config"]["n"] == (1 << 20) // 4
    assert len(out["per_rank_GBps"]) == 2 and min(out["per_rank_GBps"]) > 0
    c4 = out["c4"]
    assert c4["scaling"] == "strong" and c4["buckets"] == 48 and c4["rccl_world_size"] == 2
    assert len(c4["per_rank_GBps"]) == 2 and sum(c4["per_rank_buckets"]) == 48
    assert sorted(g["rank"] for g in shards) == [0, 1]
    a, b = (set(g["buckets"]) for g in sorted(shards, key=lambda g: g["rank"]))
    assert a and b and not (a & b)
    assert a | b == set(range(48))
    sys.path.insert(0, ROOT)
    from stellatrain_amd.shard import ShardPlan, c4_sizes
    plan = ShardPlan(c4_sizes(48, 65536, 131072), 2)
    assert sorted(a) == plan.local(0) and sorted(b) == plan.local(1)
    assert out["value"] > 0 and out["steps"] == 2


def test_bench_single_rank_headline_layout(tmp_path):
    """N = 1: the headline workload (keys x one bucket size) and the whole C4
    stream on the one rank in the c4 sub-object."""
    out, shards = _run(["--gpus", "1"], tmp_path)
    assert out["n_gpus"] == 1 and out["scaling"] == "weak" and out["rccl_world_size"] == 1
    assert out["config"]["n"] == (1 << 20) // 4
    assert out["c4"]["buckets"] == 48 and out["c4"]["per_rank_buckets"] == [48]
    assert len(shards) == 1 and len(shards[0]["buckets"]) == 48
