#!/usr/bin/env python3
"""Generate tests/golden/golden_merge.npz: the MERGE decompress at world >= 1
pinned to torch's own CPU kernels.

Producer: ``torch_merge`` below runs the exact op sequence of
``ModuleCpuOptimize::run`` under ``#if MERGE``
(engine/modules/cpu_optimize.cpp:40-72) on torch CPU tensors:

* ``merged = zeros(n)``; per rank, in rank order: ``tmp = zeros(n)``,
  ``tmp.index_put_((idx.long(),), val)`` (no accumulate), ``merged += tmp``;
* ``merged /= float(world)``;
* the union of the indices (``unique1d``: an ``unordered_set``, so its order
  is unspecified -- the golden stores the union sorted ascending);
* ``merged.index_select(0, unique_idx)``.

That block is nothing but torch CPU ops, so torch (the image's 2.10 wheel) is
the reference here, not a restatement.  Inputs are integer-generated
(``rank_streams``): per rank a stream of distinct indices, ranks sharing a
fraction of them, values from ``synth`` scaled by 1000 with some exact +0.0
and -0.0 (``+=`` onto +0.0 turns -0.0 into +0.0).  One small case repeats
indices inside a rank's stream (index_put_ without accumulate: the last
occurrence wins on the CPU's serial loop at that size).

Small cases store the whole union; the big ones (C5's 64 MiB bucket at world
2/4/8) store its size and sha256.

    python tests/golden/make_golden_merge.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from stellatrain_amd.synth import seed_for, synth  # noqa: E402

# name, n, per_rank, world, shared fraction (of per_rank, in 1/8), intra-rank duplicates, store whole
MERGE_CASES = [
    ("m_65536_w1", 65536, 655, 1, 0, False, True),
    ("m_100013_w2", 100013, 1000, 2, 4, False, True),
    ("m_100013_w3", 100013, 1000, 3, 4, False, True),
    ("m_100013_w4_disjoint", 100013, 1000, 4, 0, False, True),
    ("m_65537_w5", 65537, 3000, 5, 2, False, True),
    ("m_1m_w6", 1 << 20, 10485, 6, 4, False, True),
    ("m_1m_w8", 1 << 20, 10485, 8, 4, False, True),
    ("m_4099_w3_dups", 4099, 400, 3, 4, True, True),
    ("c5_64mib_w2", 16 << 20, 167772, 2, 4, False, False),
    ("c5_64mib_w4", 16 << 20, 167772, 4, 4, False, False),
    ("c5_64mib_w8", 16 << 20, 167772, 8, 4, False, False),
    ("c5_64mib_w8_disjoint", 16 << 20, 167772, 8, 0, False, False),
]


def _coprime_mult(n: int, salt: int) -> int:
    a = (0x9E3779B1 + 2 * salt) % n or 1
    while np.gcd(a, n) != 1:
        a += 1
    return a


def rank_streams(n: int, per_rank: int, world: int, shared8: int, dups: bool, case_seed: int):
    """world rank streams of per_rank pairs (idx u32, val f32), concatenated in
    rank order.  Indices come from one affine permutation of [0, n): the first
    h = per_rank * shared8 / 8 positions are shared by every rank, rank r owns
    the next slice after them; each stream's order is permuted by a second
    affine map.  Integer arithmetic only (identical on any numpy)."""
    h = per_rank * shared8 // 8
    own = per_rank - h
    assert h + world * own <= n
    a, b = _coprime_mult(n, case_seed), (case_seed * 7919) % n
    perm = lambda j: (a * j.astype(np.int64) + b) % n  # noqa: E731
    idx, val = [], []
    for r in range(world):
        j = np.concatenate([np.arange(h), h + r * own + np.arange(own)])
        ii = perm(j).astype(np.uint32)
        c = _coprime_mult(per_rank, case_seed + r + 1)
        ii = ii[(c * np.arange(per_rank, dtype=np.int64) + r) % per_rank]
        if dups:  # every 5th pair of the second half repeats an earlier index of the stream
            q = np.arange(per_rank // 2, per_rank, 5)
            ii[q] = ii[(q * 3) % (per_rank // 2)]
        v = synth(per_rank, seed_for(40 + r, case_seed)) * np.float32(1000)
        v[(np.arange(per_rank) % 97) == r] = np.float32(-0.0)
        v[(np.arange(per_rank) % 89) == r + 1] = np.float32(0.0)
        idx.append(ii)
        val.append(v)
    return np.concatenate(idx), np.concatenate(val)


def torch_merge(idx: np.ndarray, val: np.ndarray, per_rank: int, world: int, n: int):
    """cpu_optimize.cpp:40-72 on torch CPU tensors; returns the union sorted
    ascending with its merged values."""
    import torch
    merged = torch.zeros(int(n))
    ti = torch.from_numpy(idx.view(np.int32).copy())
    tv = torch.from_numpy(val.copy())
    parts = []
    off = 0
    for _ in range(world):
        tmp = torch.zeros(int(n))
        i = ti[off:off + per_rank]
        tmp.index_put_((i.to(torch.long),), tv[off:off + per_rank])
        parts.append(i.clone())
        merged += tmp
        off += per_rank
    merged /= float(world)
    uniq = np.unique(torch.cat(parts).numpy().view(np.uint32))  # unique1d; sorted here
    out = merged.index_select(0, torch.from_numpy(uniq.astype(np.int64)))
    return uniq, out.numpy().copy()


def digest(i: np.ndarray, v: np.ndarray) -> str:
    h = hashlib.sha256(np.ascontiguousarray(i, np.uint32).tobytes())
    h.update(np.ascontiguousarray(v, np.float32).view(np.uint32).tobytes())
    return h.hexdigest()


def main():
    import torch
    torch.set_num_threads(1)
    out, meta = {}, []
    for cs, (name, n, per_rank, world, shared8, dups, whole) in enumerate(MERGE_CASES):
        idx, val = rank_streams(n, per_rank, world, shared8, dups, cs)
        ui, uv = torch_merge(idx, val, per_rank, world, n)
        if whole:
            out[f"{name}/idx"] = ui
            out[f"{name}/val"] = uv
        meta.append({"name": name, "n": n, "per_rank": per_rank, "world": world, "shared8": shared8, "dups": dups,
                     "case_seed": cs, "whole": whole, "union": int(ui.size), "sha256": digest(ui, uv)})
        print(name, ui.size)
    np.savez_compressed(os.path.join(HERE, "golden_merge.npz"), **out)
    with open(os.path.join(HERE, "manifest_merge.json"), "w") as f:
        json.dump({"producer": "torch CPU ops of cpu_optimize.cpp:40-72 (zeros, index_put_, +=, /= float(world), "
                               "index_select), torch " + torch.__version__, "merge": meta}, f, indent=1)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    main()
