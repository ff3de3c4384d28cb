"""thresholdv16 launches need no workgroup co-residency.

Every wait in the scan launch points at a chunk an already-running workgroup
took (slots 0 and 1 come from the call's counter too), and the regime-B fill
is a separate launch with no inter-workgroup waits.  So four launches in
flight at once, or foreign kernels holding CUs on another stream, may slow a
launch down but never stall it: outputs stay bit-exact and the device failure
word stays clean.  Each case runs once, in a child process (the in-flight
setting is read once per process).
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _child(streams: int, gemm: int, inflight: int):
    env = dict(os.environ, STG_TV16_INFLIGHT=str(inflight))
    r = subprocess.run([sys.executable, os.path.join(HERE, "inflight_child.py"), str(streams), str(gemm)],
                       capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["ok"] and out["buckets_checked"] == 4 * 4 * streams
    return out


def test_four_launches_in_flight(gpu):
    _child(4, 0, 4)


def test_foreign_gemm_on_another_stream(gpu):
    _child(2, 6, 2)
