#!/usr/bin/env python3
"""Generate tests/golden/golden_gather.npz from the REFERENCE add_arrays.

Producer: oracle/_ref/libstg_ref_gather.so -- misc/array_util.h compiled in
place from /root/reference with -g -O3 -march=broadwell by oracle/Makefile,
driven by oracle/ref_gather_driver.cpp through the per-rank slices of
ModuleCpuGather::run (engine/modules/cpu_gather.cpp:59-87).  Every local rank
of the node runs its slice; the stored array is grad[0] afterwards.  Inputs are
regenerated from synth(n, seed_for(71 + i, 0)) (grads, D1) and
synth(n, seed_for(70, 0), D2) (residual).

    python tests/golden/make_golden_gather.py
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.oracle import REF_SO, build  # noqa: E402
from stellatrain_amd.synth import D1, D2, seed_for, synth  # noqa: E402

GATHER_CASES = [("gather_100013_g4", 100013, 4), ("gather_65536_g8", 65536, 8), ("gather_1000_g2", 1000, 2),
                ("gather_33_g3", 33, 3), ("gather_4099_g1", 4099, 1)]


def inputs(n, g):
    grads = [synth(n, seed_for(71 + i, 0), D1) for i in range(g)]
    return grads, synth(n, seed_for(70, 0), D2)


def main():
    build(ref=True)
    lib = C.CDLL(os.path.join(os.path.dirname(REF_SO), "libstg_ref_gather.so"))
    lib.ref_gather_add.argtypes = [np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS"),
                                   np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS"),
                                   C.POINTER(C.c_void_p), C.c_int, C.c_int64, C.c_int]
    out, meta = {}, []
    for name, n, g in GATHER_CASES:
        grads, resid = inputs(n, g)
        ptrs = (C.c_void_p * g)(*[x.ctypes.data for x in grads])
        for r in range(g):
            lib.ref_gather_add(grads[0], resid, ptrs, g, n, r)
        out[f"{name}/grad0"] = grads[0]
        meta.append({"name": name, "n": n, "num_gpus": g})
    np.savez_compressed(os.path.join(HERE, "golden_gather.npz"), **out)
    with open(os.path.join(HERE, "manifest_gather.json"), "w") as f:
        json.dump({"producer": "reference misc/array_util.h add_arrays compiled in place (oracle/Makefile)",
                   "flags": "-std=c++17 -g -O3 -march=broadwell", "gather": meta}, f, indent=1)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    main()
