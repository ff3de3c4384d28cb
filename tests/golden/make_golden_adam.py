#!/usr/bin/env python3
"""Generate tests/golden/golden_adam.npz from the REFERENCE sparse Adam itself.

Producer: oracle/_ref/libstg_ref_adam.so -- the reference's optim/adam.cpp
compiled in place from /root/reference with -g -O3 -march=broadwell
(backend/CMakeLists.txt:28-32) by oracle/Makefile, driven through
oracle/ref_adam_driver.cpp.  The sparse gradients are the reference
thresholdv16 codec's own output (oracle/_ref/libstg_ref.so) on synthetic
buckets, so the index order is the codec's (it matters for amsgrad's running
vmax, adam.cpp:71).

Stored: param after the last step, the m / v state arrays, vmax and tick.

    python tests/golden/make_golden_adam.py
"""
from __future__ import annotations

import ctypes as C
import json
import os
import platform
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.oracle import REF_SO, Reference, build  # noqa: E402
from stellatrain_amd.synth import D1, seed_for, synth  # noqa: E402

# (name, n, k, lr, b1, b2, eps, weight_decay, amsgrad, maximize, steps)
ADAM_CASES = [
    ("adam_default", 100013, 1000, 1e-3, 0.9, 0.999, 1e-8, 0.0, False, False, 4),
    ("adam_amsgrad_wd", 100013, 1000, 1e-2, 0.9, 0.999, 1e-8, 1e-2, True, False, 4),
    ("adam_maximize", 65536, 655, 5e-3, 0.8, 0.99, 1e-6, 0.0, False, True, 3),
    ("adam_amsgrad_small", 4103, 40, 1e-1, 0.5, 0.9, 1e-4, 0.0, True, False, 5),
]
SEED_BUCKET = 29


def gen_adam(out):
    lib = C.CDLL(os.path.join(os.path.dirname(REF_SO), "libstg_ref_adam.so"))
    f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
    u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
    lib.ref_adam_new.restype = C.c_void_p
    lib.ref_adam_new.argtypes = [C.c_float] * 5 + [C.c_int, C.c_int]
    lib.ref_adam_apply.argtypes = [C.c_void_p, C.c_char_p, f32p, C.c_uint32, f32p, u32p, C.c_uint32]
    lib.ref_adam_state.restype = C.c_int
    lib.ref_adam_state.argtypes = [C.c_void_p, C.c_char_p, f32p, f32p, C.c_uint32, C.POINTER(C.c_float)]
    lib.ref_adam_free.argtypes = [C.c_void_p]
    ref = Reference()
    meta = []
    for (name, n, k, lr, b1, b2, eps, wd, ams, maxi, steps) in ADAM_CASES:
        o = lib.ref_adam_new(lr, b1, b2, eps, wd, int(ams), int(maxi))
        h = ref.tv16_new()
        param = synth(n, seed_for(SEED_BUCKET, 99), D1) * np.float32(1000.0)
        for s in range(steps):
            g = synth(n, seed_for(SEED_BUCKET, s), D1)
            cnt, idx, val = ref.tv16_compress(h, "p", g, k)
            lib.ref_adam_apply(o, b"p", param, n, np.ascontiguousarray(val[:cnt]),
                               np.ascontiguousarray(idx[:cnt]), cnt)
        m, v, vmax = np.zeros(n, np.float32), np.zeros(n, np.float32), C.c_float()
        tick = lib.ref_adam_state(o, b"p", m, v, n, C.byref(vmax))
        out[f"{name}/param"] = param
        out[f"{name}/m"] = m
        out[f"{name}/v"] = v
        meta.append({"name": name, "n": n, "k": k, "lr": lr, "b1": b1, "b2": b2, "eps": eps,
                     "weight_decay": wd, "amsgrad": ams, "maximize": maxi, "steps": steps,
                     "seed_bucket": SEED_BUCKET, "param_init": "synth(n, seed_for(29, 99), D1) * 1000",
                     "grad_codec": "thresholdv16", "tick": tick,
                     "vmax_bits": int(np.float32(vmax.value).view(np.uint32))})
        lib.ref_adam_free(o)
        ref.tv16_free(h)
    return meta


def main():
    build(ref=True)
    gxx = subprocess.run(["g++", "--version"], capture_output=True, text=True).stdout.splitlines()[0]
    manifest = {"producer": "reference backend/src/optim/adam.cpp compiled in place (oracle/Makefile)",
                "flags": "-std=c++17 -g -O3 -march=broadwell", "compiler": gxx, "host": platform.machine(),
                "generator": "stellatrain_amd/synth.py (splitmix64 Irwin-Hall, SURVEY 8(c))"}
    out: dict[str, np.ndarray] = {}
    manifest["adam"] = gen_adam(out)
    np.savez_compressed(os.path.join(HERE, "golden_adam.npz"), **out)
    with open(os.path.join(HERE, "manifest_adam.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("wrote", len(out), "arrays;", os.path.getsize(os.path.join(HERE, "golden_adam.npz")) >> 10, "KiB")


if __name__ == "__main__":
    main()
