"""A bounded wait that gives up, end to end ("device
failures surface"): a debug switch makes Top-k's first emission unit
withhold its counts, so the later units' look-backs run out their bound; the launch
must poison its count, set the sticky failure word, and the host entry points
must raise.  Runs in a child process (the switch is read once per process)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_lookback_gives_up():
    env = dict(os.environ, STG_DEBUG_TK_WITHHOLD="1")
    r = subprocess.run([sys.executable, os.path.join(HERE, "timeout_child.py")], env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["count"] == 0xffffffff, out
    assert out["check"] != "ok" and out["compress"] != "ok", out
