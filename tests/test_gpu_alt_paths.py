"""The codecs' opt-in launch shapes against the oracle, each in a child
process (tests/alt_path_child.py; the switches are read once per process):
Top-k's finish inside the stream launch (STG_TK2_FIN=1) and threshold-v's
chunk launches (STG_TV_PASS=0).  DESIGN.md section 4 has their measurements
against the default shapes."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _child(**env):
    e = dict(os.environ, **env)
    r = subprocess.run([sys.executable, os.path.join(HERE, "alt_path_child.py")], capture_output=True, text=True,
                       timeout=110, env=e)
    assert r.returncode == 0, r.stderr[-4000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


def test_topk_finish_in_stream(gpu):
    out = _child(STG_TK2_FIN="1")
    assert out["topk_calls"] == 56
    for mode, (hits, sel, in_stream, tk_one_ran) in out["topk_words"].items():
        # every hit finished inside the stream launch; tk_one's workgroups ran
        # only for the calls that took the select's way
        assert hits >= 10 and in_stream == hits and sel >= 4, (mode, out)


def test_thresholdv_chunk_launches(gpu):
    out = _child(STG_TV_PASS="0")
    assert out["tv_calls"] == 25
