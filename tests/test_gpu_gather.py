"""GPU parity of the intra-node gather-add (ModuleCpuGather::run,
engine/modules/cpu_gather.cpp:59-87) through ``stg_gather_add_device``:
against the reference's own add_arrays goldens (tests/golden/
golden_gather.npz) and the oracle on slices of every phase (the vector path's
scalar head and tail).  Bit-exact.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import pytest

from stellatrain_amd.synth import D1, D2, seed_for, synth

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MANIFEST_GATHER = json.load(open(os.path.join(GOLD, "manifest_gather.json")))


@pytest.mark.parametrize("case", MANIFEST_GATHER["gather"], ids=lambda c: c["name"])
def test_gather_add_matches_reference_goldens(gpu, case):
    import torch
    from stellatrain_amd import gather_add
    sys.path.insert(0, GOLD)
    from make_golden_gather import inputs
    n, g = case["n"], case["num_gpus"]
    grads, resid = inputs(n, g)
    dg = [torch.from_numpy(x).to(gpu) for x in grads]
    dr = torch.from_numpy(resid).to(gpu)
    for r in range(g):  # every local rank's slice (on one device here)
        gather_add(dg, dr, r)
    ref = np.load(os.path.join(GOLD, "golden_gather.npz"))[f"{case['name']}/grad0"]
    assert np.array_equal(dg[0].cpu().numpy().view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("n,g,offs", [(1 << 20, 8, (0, 0, 0)), (100003, 4, (1, 1, 1)), (65541, 3, (2, 0, 1)),
                                      (9, 5, (3, 3, 3))])
def test_gather_add_phases(gpu, oracle, n, g, offs):
    """Sources at equal and at differing 16-byte phases (vector path with a
    scalar head, and the all-scalar fallback), no residual on one pass."""
    import torch
    from stellatrain_amd import gather_add
    o_dst, o_res, o_src = offs
    grads = [synth(n, seed_for(80 + i, 1), D1 if i % 2 else D2) for i in range(g)]
    resid = synth(n, seed_for(79, 1), D2)
    base = [torch.zeros(n + 4, dtype=torch.float32, device=gpu) for _ in range(g + 1)]
    dg = []
    for i in range(g):
        o = o_dst if i == 0 else o_src
        base[i][o:o + n].copy_(torch.from_numpy(grads[i]))
        dg.append(base[i][o:o + n])
    base[g][o_res:o_res + n].copy_(torch.from_numpy(resid))
    dr = base[g][o_res:o_res + n]
    og = [x.copy() for x in grads]
    for r in range(g):
        oracle.gather_add(og, resid, r)
        gather_add(dg, dr, r)
    assert np.array_equal(dg[0].cpu().numpy().view(np.uint32), og[0].view(np.uint32))
    # a second pass without the residual term
    og2 = [x.copy() for x in og]
    zero = np.zeros(n, np.float32)
    for r in range(g):
        oracle.gather_add(og2, zero, r)  # +0.0 residual == no residual for these nonzero inputs
        gather_add(dg, None, r)
    got = dg[0].cpu().numpy()
    nz = og2[0] != 0
    assert np.array_equal(got[nz].view(np.uint32), og2[0][nz].view(np.uint32))
