"""GPU parity of the sparse Adam apply (optim/adam.cpp:19-86) through the C-ABI
(``stg_adam_optimize_raw_device``).

* Against the reference's own goldens (tests/golden/golden_adam.npz, made by
  make_golden_adam.py from the reference compiled in place): the same codec
  streams replayed through the HIP path give bit-identical param, m, v, vmax
  and tick.
* Against the pinned oracle restatement on shuffled index orders and tile
  counts past one scan workgroup (amsgrad's running vmax is order dependent,
  adam.cpp:71), with a device-side grad count, and on repeated names.

All comparisons are bit-exact (fp32 bit patterns).
"""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

from stellatrain_amd.synth import D1, D2, seed_for, synth

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MANIFEST_ADAM = json.load(open(os.path.join(GOLD, "manifest_adam.json")))


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _opts(case):
    return dict(lr=case["lr"], b1=case["b1"], b2=case["b2"], eps=case["eps"], weight_decay=case["weight_decay"],
                amsgrad=case["amsgrad"], maximize=case["maximize"])


@pytest.mark.parametrize("case", MANIFEST_ADAM["adam"], ids=lambda c: c["name"])
def test_adam_matches_reference_goldens(gpu, oracle, case):
    import torch
    from stellatrain_amd import SparseAdam
    arr = np.load(os.path.join(GOLD, "golden_adam.npz"))
    n, k = case["n"], case["k"]
    adam = SparseAdam(**_opts(case))
    h = oracle.tv16_new()
    pg = torch.from_numpy(synth(n, seed_for(case["seed_bucket"], 99)) * np.float32(1000.0)).to(gpu)
    for s in range(case["steps"]):
        g = synth(n, seed_for(case["seed_bucket"], s))
        cnt, idx, val = oracle.tv16_compress(h, "p", g, k)  # == the reference stream (pinned)
        adam.optimize_raw(pg, "p", torch.from_numpy(np.ascontiguousarray(val[:cnt])).to(gpu),
                          torch.from_numpy(np.ascontiguousarray(idx[:cnt]).view(np.int32)).to(gpu))
    name = case["name"]
    assert np.array_equal(_bits(pg.cpu().numpy()), _bits(arr[f"{name}/param"]))
    m, v, vmax, tick = adam.state("p", n)
    assert np.array_equal(_bits(m), _bits(arr[f"{name}/m"]))
    assert np.array_equal(_bits(v), _bits(arr[f"{name}/v"]))
    assert int(np.float32(vmax).view(np.uint32)) == case["vmax_bits"] and tick == case["tick"]
    oracle.tv16_free(h)


ADAM_CASES = [
    # name, n, k, opts
    ("default", 100013, 1000, dict()),
    ("amsgrad", 1 << 20, 300000, dict(lr=1e-2, amsgrad=True)),  # 293 tiles: scan past one workgroup
    ("amsgrad_wd_max", 262144, 2621, dict(lr=5e-3, weight_decay=1e-2, amsgrad=True, maximize=True)),
    ("b_eps", 4099, 41, dict(lr=0.1, b1=0.5, b2=0.9, eps=1e-4)),
]


@pytest.mark.parametrize("name,n,k,opts", ADAM_CASES, ids=[c[0] for c in ADAM_CASES])
def test_adam_apply_parity(gpu, oracle, name, n, k, opts):
    import torch
    from stellatrain_amd import SparseAdam
    param0 = synth(n, seed_for(37, 99)) * np.float32(1000)
    po = param0.copy()
    pg = torch.from_numpy(param0.copy()).to(gpu)
    ho = oracle.adam_new(**opts)
    adam = SparseAdam(**opts)
    rng = np.random.default_rng(11)
    for step in range(4):
        # steps 0-1 reuse one shuffled index set (moment re-use); 2-3 a fresh one
        if step % 2 == 0:
            gidx = rng.choice(n, k, replace=False).astype(np.uint32)
        g = synth(k, seed_for(41, step), D2) * np.float32(100)
        oracle.adam_apply(ho, "fc@weight", po, g, gidx)
        adam.optimize_raw(pg, "fc@weight", torch.from_numpy(g).to(gpu), torch.from_numpy(gidx.view(np.int32)).to(gpu))
        assert np.array_equal(_bits(pg.cpu().numpy()), _bits(po)), f"param differs at step {step}"
    mo, vo, vmo, to = oracle.adam_state(ho, "fc@weight", n)
    mg, vg, vmg, tg = adam.state("fc@weight", n)
    assert np.array_equal(_bits(mg), _bits(mo)) and np.array_equal(_bits(vg), _bits(vo))
    assert _bits(vmg) == _bits(vmo) and tg == to
    oracle.adam_free(ho)


def test_adam_device_count_and_names(gpu, oracle):
    """grad_len is a capacity; the device count (as the codecs write it) bounds
    the update.  Two names keep separate state and ticks."""
    import torch
    from stellatrain_amd import SparseAdam
    n, cap, cnt = 65536, 4096, 3001
    opts = dict(lr=1e-2, amsgrad=True)
    ho, adam = oracle.adam_new(**opts), SparseAdam(**opts)
    rng = np.random.default_rng(5)
    pa0 = synth(n, seed_for(43, 1)) * np.float32(10)
    pb0 = synth(n, seed_for(43, 2)) * np.float32(10)
    pa, pb = pa0.copy(), pb0.copy()
    ga, gb = torch.from_numpy(pa0.copy()).to(gpu), torch.from_numpy(pb0.copy()).to(gpu)
    dcnt = torch.tensor([cnt], dtype=torch.int32, device=gpu)
    for step in range(3):
        gidx = rng.choice(n, cap, replace=False).astype(np.uint32)
        g = synth(cap, seed_for(47, step), D1) * np.float32(1000)
        oracle.adam_apply(ho, "a", pa, g[:cnt], gidx[:cnt])
        adam.optimize_raw(ga, "a", torch.from_numpy(g).to(gpu), torch.from_numpy(gidx.view(np.int32)).to(gpu),
                          grad_len=cap, d_grad_len=dcnt)
        if step < 2:
            oracle.adam_apply(ho, "b", pb, g, gidx)
            adam.optimize_raw(gb, "b", torch.from_numpy(g).to(gpu), torch.from_numpy(gidx.view(np.int32)).to(gpu))
    assert np.array_equal(_bits(ga.cpu().numpy()), _bits(pa))
    assert np.array_equal(_bits(gb.cpu().numpy()), _bits(pb))
    for nm in ("a", "b"):
        mo, vo, vmo, to = oracle.adam_state(ho, nm, n)
        mg, vg, vmg, tg = adam.state(nm, n)
        assert np.array_equal(_bits(mg), _bits(mo)) and np.array_equal(_bits(vg), _bits(vo))
        assert _bits(vmg) == _bits(vmo) and tg == to
    assert adam.state("never", n) is None
    oracle.adam_free(ho)
