"""Pin the CPU oracle (oracle/stg_oracle.cpp) to golden vectors produced by the
reference's own codec (tests/golden/make_golden.py, oracle/_ref build).

Runs everywhere (CPU only); the GPU parity tests then compare the HIP path
against this pinned oracle.
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np
import pytest

from stellatrain_amd.synth import seed_for, synth

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
MANIFEST = json.load(open(os.path.join(GOLD, "manifest.json")))
ARR = np.load(os.path.join(GOLD, "golden.npz"))
MANIFEST_ADAM = json.load(open(os.path.join(GOLD, "manifest_adam.json")))
ARR_ADAM = np.load(os.path.join(GOLD, "golden_adam.npz"))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def f32bits(x):
    return int(np.float32(x).view(np.uint32))


@pytest.mark.parametrize("case", MANIFEST["tv16"], ids=lambda c: c["name"])
def test_tv16_oracle_matches_reference(oracle, case):
    h = oracle.tv16_new()
    name = case["name"]
    for it in range(case["iters"]):
        src = synth(case["n"], seed_for(case["seed_bucket"], it), case["dist"], case["param"])
        cnt, idx, val = oracle.tv16_compress(h, case["key"], src, case["k"])
        assert cnt == ARR[f"{name}/counts"][it]
        t, inc = oracle.tv16_state(h, case["key"])
        assert f32bits(t) == ARR[f"{name}/t_bits"][it]
        assert f32bits(inc) == ARR[f"{name}/inc_bits"][it]
        if case["full"]:
            np.testing.assert_array_equal(idx[:cnt], ARR[f"{name}/it{it}/idx"])
            np.testing.assert_array_equal(val[:cnt].view(np.uint32), ARR[f"{name}/it{it}/val"].view(np.uint32))
        assert sha(idx[:cnt]) + ":" + sha(val[:cnt].view(np.uint32)) == case["hashes"][it]
    oracle.tv16_free(h)


@pytest.mark.parametrize("case", MANIFEST["tv"], ids=lambda c: c["name"])
def test_tv_oracle_matches_reference(oracle, case):
    h = oracle.tv_new()
    name = case["name"]
    for it in range(case["iters"]):
        src = synth(case["n"], seed_for(case["seed_bucket"], it), case["dist"], case["param"])
        cnt, idx, val = oracle.tv_compress(h, 1, src, case["k"])
        assert cnt == ARR[f"{name}/counts"][it]
        assert f32bits(oracle.tv_state(h, 1)) == ARR[f"{name}/t_bits"][it]
        if case["full"]:
            np.testing.assert_array_equal(idx[:cnt], ARR[f"{name}/it{it}/idx"])
            np.testing.assert_array_equal(val[:cnt].view(np.uint32), ARR[f"{name}/it{it}/val"].view(np.uint32))
        assert sha(idx[:cnt]) + ":" + sha(val[:cnt].view(np.uint32)) == case["hashes"][it]
    oracle.tv_free(h)


@pytest.mark.parametrize("case", MANIFEST["topk"], ids=lambda c: c["name"])
def test_topk_oracle_matches_reference(oracle, case):
    """bug-compat top-k, including libstdc++ nth_element partition order."""
    src = synth(case["n"], seed_for(case["seed_bucket"], 0), case["dist"], case["param"])
    cnt, idx, val = oracle.topk_compress(src, case["k"], bug_compat=True)
    assert cnt == case["count"]
    np.testing.assert_array_equal(idx, ARR[f"{case['name']}/idx"])
    np.testing.assert_array_equal(val.view(np.uint32), ARR[f"{case['name']}/val"].view(np.uint32))


@pytest.mark.parametrize("case", MANIFEST["sgd"], ids=lambda c: c["name"])
def test_sgd_oracle_matches_reference(oracle, case):
    n, k = case["n"], case["k"]
    o = oracle.sgd_new(case["lr"], case["momentum"], case["dampening"], case["weight_decay"], case["nesterov"])
    h = oracle.tv16_new()
    param = synth(n, seed_for(case["seed_bucket"], 99)) * np.float32(1000.0)
    for s in range(case["steps"]):
        g = synth(n, seed_for(case["seed_bucket"], s))
        cnt, idx, val = oracle.tv16_compress(h, "p", g, k)
        oracle.sgd_apply(o, "p", param, val[:cnt], idx[:cnt])
    np.testing.assert_array_equal(param.view(np.uint32), ARR[f"{case['name']}/param"].view(np.uint32))
    key = f"{case['name']}/momentum"
    if key in ARR.files:
        m = oracle.sgd_momentum(o, "p", n)
        np.testing.assert_array_equal(m.view(np.uint32), ARR[key].view(np.uint32))
    oracle.sgd_free(o)


@pytest.mark.parametrize("case", MANIFEST_ADAM["adam"], ids=lambda c: c["name"])
def test_adam_oracle_matches_reference(oracle, case):
    """optim/adam.cpp:19-86 restated; param, m, v, vmax and tick bit-exact."""
    n, k = case["n"], case["k"]
    o = oracle.adam_new(case["lr"], case["b1"], case["b2"], case["eps"], case["weight_decay"], case["amsgrad"],
                        case["maximize"])
    h = oracle.tv16_new()
    param = synth(n, seed_for(case["seed_bucket"], 99)) * np.float32(1000.0)
    for s in range(case["steps"]):
        g = synth(n, seed_for(case["seed_bucket"], s))
        cnt, idx, val = oracle.tv16_compress(h, "p", g, k)
        oracle.adam_apply(o, "p", param, val[:cnt], idx[:cnt])
    name = case["name"]
    np.testing.assert_array_equal(param.view(np.uint32), ARR_ADAM[f"{name}/param"].view(np.uint32))
    m, v, vmax, tick = oracle.adam_state(o, "p", n)
    np.testing.assert_array_equal(m.view(np.uint32), ARR_ADAM[f"{name}/m"].view(np.uint32))
    np.testing.assert_array_equal(v.view(np.uint32), ARR_ADAM[f"{name}/v"].view(np.uint32))
    assert f32bits(vmax) == case["vmax_bits"] and tick == case["tick"]
    oracle.adam_free(o)
    oracle.tv16_free(h)


def test_goldens_cover_both_regimes():
    """The fixtures contain AIMD increases (regime A) and decreases (regime B)."""
    ups = downs = 0
    for c in MANIFEST["tv16"]:
        t = ARR[f"{c['name']}/t_bits"].view(np.float32)
        d = np.diff(t.astype(np.float64))
        ups += int((d > 0).sum())
        downs += int((d < 0).sum())
    assert ups > 10 and downs > 10


MANIFEST_GATHER = json.load(open(os.path.join(GOLD, "manifest_gather.json")))


@pytest.mark.parametrize("case", MANIFEST_GATHER["gather"], ids=lambda c: c["name"])
def test_gather_add_oracle_matches_reference(oracle, case):
    """cpu_gather.cpp:59-87 + array_util.h add_arrays, every local rank's slice."""
    import sys
    sys.path.insert(0, GOLD)
    from make_golden_gather import inputs
    n, g = case["n"], case["num_gpus"]
    grads, resid = inputs(n, g)
    for r in range(g):
        oracle.gather_add(grads, resid, r)
    ref = np.load(os.path.join(GOLD, "golden_gather.npz"))[f"{case['name']}/grad0"]
    np.testing.assert_array_equal(grads[0].view(np.uint32), ref.view(np.uint32))


def test_gather_slices_partition(oracle):
    """The local ranks' slices tile [0, n) exactly (cpu_gather.cpp:59-61)."""
    for n in (0, 1, 7, 33, 100013, 1 << 24):
        for g in range(1, 9):
            cur = 0
            for r in range(g):
                a, b = oracle.gather_slice(n, r, g)
                assert a == cur and b >= a
                cur = b
            assert cur == n



# MERGE decompress at world >= 1 pinned to torch's own CPU kernels
# (tests/golden/make_golden_merge.py runs cpu_optimize.cpp:40-72's op sequence)
from merge_golden import MANIFEST_MERGE, merge_case_check, merge_case_inputs  # noqa: E402


@pytest.mark.parametrize("case", MANIFEST_MERGE["merge"], ids=lambda c: c["name"])
def test_merge_oracle_matches_torch(oracle, case):
    idx, val = merge_case_inputs(case)
    oi, ov = oracle.merge_decompress(idx, val, case["per_rank"], case["world"], case["n"])
    merge_case_check(case, oi, ov)
