"""The torch-pinned MERGE decompress goldens (tests/golden/make_golden_merge.py):
inputs regenerated from the manifest, outputs compared bit for bit."""
from __future__ import annotations

import json
import os
import sys

import numpy as np

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLD)
from make_golden_merge import digest, rank_streams  # noqa: E402

MANIFEST_MERGE = json.load(open(os.path.join(GOLD, "manifest_merge.json")))
ARR_MERGE = np.load(os.path.join(GOLD, "golden_merge.npz"))


def merge_case_inputs(case):
    return rank_streams(case["n"], case["per_rank"], case["world"], case["shared8"], case["dups"], case["case_seed"])


def merge_case_check(case, out_idx, out_val):
    """out_idx / out_val: the union in any order; compared sorted, bit for bit."""
    o = np.argsort(np.asarray(out_idx, np.uint32), kind="stable")
    gi, gv = np.asarray(out_idx, np.uint32)[o], np.asarray(out_val, np.float32)[o]
    assert gi.size == case["union"]
    if case["whole"]:
        np.testing.assert_array_equal(gi, ARR_MERGE[f"{case['name']}/idx"])
        np.testing.assert_array_equal(gv.view(np.uint32), ARR_MERGE[f"{case['name']}/val"].view(np.uint32))
    assert digest(gi, gv) == case["sha256"]
