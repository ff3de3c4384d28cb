"""Every way the regime-B heap fill orders equal sums gives the reference's stream.

tv16fill.hip orders a regime-B bucket's heap pops one of four ways: no two
popped sums tie (sum order), ties ordered by right-first pre-order of their
start positions (when its two checks pass), the shadow heap, or the literal
make_heap / pop_heap in global memory.  A one-bucket call's finish
(tv16lfin.h) first lets its rankers order the fill in parallel by the same
right-first rule and falls back to that orderer when they cannot prove it.
A bucket whose window below t misses the pops (a drop of the gradient scale)
is ordered by the crew (tv16wide.h): extra workgroups of the fill launch list
its top candidates again and the leader orders them; the leader also takes the
orderer's calls its LDS paths cannot.  STG_DEBUG_TV16_FILL forces the heavier
ways, so each is checked against the oracle on the same tie-heavy AIMD
sequences (one-bucket calls and a batched launch, each ending in a 100x scale
drop); the path counters show which way ran.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _child(mode: int, **extra):
    env = dict(os.environ, STG_DEBUG_TV16_FILL=str(mode), **extra)
    r = subprocess.run([sys.executable, os.path.join(HERE, "fill_mode_child.py")],
                       capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


def test_production_order(gpu):
    """One-bucket calls: the scan launch's finish (tv16lf2.h) ranks the
    regime-B fills; D1's regime-B calls tie among the pops.  The scale drops
    are window misses: the fill launch's crew orders them, never the literal
    heap."""
    out = _child(0)
    plain, tied, viol, notake = out["lfin"]
    assert out["scan_ranked"][1] > 0, out  # ranked with ties in the scan launch
    assert out["stale"] == 0, out  # no list entry without its call's tag (tv16lf2.h freshness check)
    assert out["paths"][3] == 0, out  # never the literal heap
    leader, crew, leader_lit, crew_lit = out["wide"]
    assert crew > 0 and leader_lit == 0 and crew_lit == 0, out


@pytest.mark.parametrize("env", [{"STG_TV16_LF2": "0"}, {"STG_LF2_SKIP": "1"}, {"STG_LF2_SKIP": "4"},
                                 {"STG_LF2_SKIP": "5"}],
                         ids=["lfin_only", "scan_rankers_give_up", "scan_workers_give_up", "scan_lists_stale"])
def test_production_order_fill_finish(gpu, env):
    """The fill launch's finish (tv16lfin.h): with the scan's finish off, or
    with its rankers / workers giving up (STG_LF2_SKIP), the fill launch's
    rankers order the regime-B fills (with ties), bit-exact as before.  With
    STG_LF2_SKIP=5 the scan tags its lists with a wrong call tag: the finish's
    freshness check must send every call with qualifying lines to the fill
    launch (debug word 31) and the streams stay bit-exact."""
    out = _child(0, **env)
    if env.get("STG_LF2_SKIP") == "5":
        assert out["stale"] > 0, out
    else:
        assert out["stale"] == 0, out
    plain, tied, viol, notake = out["lfin"]
    assert tied > 0, out
    assert out["paths"][3] == 0, out  # never the literal heap
    leader, crew, leader_lit, crew_lit = out["wide"]
    assert crew > 0 and leader_lit == 0 and crew_lit == 0, out


def test_production_order_orderer_alone(gpu):
    """The one-bucket finish without rankers: its last workgroup runs the
    orderer (tv16fill.hip) on every regime-B call."""
    out = _child(0, STG_TV16_LFIN_RANKERS="0", STG_TV16_LF2="0")
    none, by_start, shadow, literal = out["paths"]
    assert by_start > 0 and literal == 0, out
    assert out["lfin"] == [0, 0, 0, 0], out


def test_production_order_batched_lone_fill(gpu):
    """The batched scan for a lone bucket (STG_TV16_LFIN=0): its fill with
    helper workgroups."""
    out = _child(0, STG_TV16_LFIN="0")
    none, by_start, shadow, literal = out["paths"]
    assert by_start > 0 and literal == 0, out


def test_shadow_heap_order(gpu):
    out = _child(1)
    none, by_start, shadow, literal = out["paths"]
    assert by_start == 0 and shadow > 0 and literal == 0, out


def test_literal_heap_order(gpu):
    out = _child(2)
    none, by_start, shadow, literal = out["paths"]
    assert by_start == 0 and shadow == 0 and literal > 0, out
    assert out["wide"] == [0, 0, 0, 0], out


def test_leader_order(gpu):
    """The leader over the window list on every regime-B call the window
    holds (the orderer's fast paths skipped); the crew for the misses."""
    out = _child(3)
    none, by_start, shadow, literal = out["paths"]
    leader, crew, leader_lit, crew_lit = out["wide"]
    assert by_start == 0 and shadow == 0 and literal == 0, out
    assert leader > 0 and crew > 0 and leader_lit == 0 and crew_lit == 0, out


def test_crew_order(gpu):
    """The crew on every regime-B bucket (window or not)."""
    out = _child(4)
    none, by_start, shadow, literal = out["paths"]
    leader, crew, leader_lit, crew_lit = out["wide"]
    assert literal == 0 and leader == 0 and crew > 0 and crew_lit == 0, out
