#!/usr/bin/env python3
"""Generate tests/golden/*.npz from the REFERENCE codec itself.

Producer: oracle/_ref/libstg_ref.so and libstg_ref_sgd.so -- the reference's
backend/src/compress/{thresholdv16,thresholdv,topk}.cpp, engine/threadpool.cpp
and optim/sgd.cpp compiled in place from /root/reference with the reference's
RelWithDebInfo flags (-g -O3 -march=broadwell, backend/CMakeLists.txt:28-32)
by oracle/Makefile.  Only this container has /root/reference; the GPU box gets
the committed fixtures.

Inputs are not stored: they are regenerated bit-exactly from
(n, seed, dist, param) by stellatrain_amd/synth.py (integer-only generator,
SURVEY.md 8(c)).  Outputs: counts, per-call AIMD threshold bits, full
(idx, val) streams for the small cases, sha256 of the streams for the large
ones.

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import ctypes as C
import hashlib
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
from stellatrain_amd.synth import D1, D2, D3, seed_for, synth  # noqa: E402

# (name, n, k, dist, param, iters, full_arrays)
TV16_CASES = [
    ("tv16_64k_d1", 65536, 655, D1, 0, 16, True),
    ("tv16_100013_d1", 100013, 1007, D1, 0, 16, True),
    ("tv16_100013_d2", 100013, 1007, D2, 0, 16, True),
    ("tv16_100013_d3_90", 100013, 1007, D3, 9000, 12, True),
    ("tv16_64k_d3_9995", 65536, 655, D3, 9995, 12, True),
    ("tv16_4103_d1", 4103, 40, D1, 0, 16, True),
    ("tv16_1000_k7", 1000, 7, D1, 0, 16, True),
    ("tv16_33_k3", 33, 3, D1, 0, 12, True),
    ("tv16_1m3_d1", 1000003, 10000, D1, 0, 16, False),
    ("tv16_1m_k9999", 1000000, 9999, D1, 0, 12, False),
]
TV_CASES = [
    ("tv_100013_d1", 100013, 100, D1, 0, 16, True),
    ("tv_100013_d2", 100013, 100, D2, 0, 16, True),
    ("tv_5000_k4999", 5000, 4999, D1, 0, 8, True),
    ("tv_1m_d1", 1 << 20, 1048, D1, 0, 16, False),
]
TOPK_CASES = [
    ("topk_100013", 100013, 1000, D1, 0),
    ("topk_4099", 4099, 41, D1, 0),
    ("topk_1m", 1 << 20, 10485, D2, 0),
]
SGD_CASES = [  # (name, n, k, lr, momentum, dampening, wd, nesterov, steps)
    ("sgd_m09", 100013, 1000, 0.1, 0.9, 0.0, 0.0, False, 3),
    ("sgd_nesterov_wd", 100013, 1000, 0.05, 0.9, 0.1, 1e-4, True, 3),
    ("sgd_plain", 65536, 655, 0.01, 0.0, 0.0, 0.0, False, 2),
]


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def gen_codec(ref, cases, kind, out):
    meta = []
    for (name, n, k, dist, param, iters, full) in cases:
        h = ref.tv16_new() if kind == "tv16" else ref.tv_new()
        counts, tbits, incbits, hashes = [], [], [], []
        for it in range(iters):
            src = synth(n, seed_for(17, it), dist, param)
            if kind == "tv16":
                cnt, idx, val = ref.tv16_compress(h, "5@weight", src, k)
                t, inc = ref.tv16_state(h, "5@weight")
            else:
                cnt, idx, val = ref.tv_compress(h, 1, src, k)
                t, inc = ref.tv_state(h, 1), 0.0
            counts.append(cnt)
            tbits.append(int(np.float32(t).view(np.uint32)))
            incbits.append(int(np.float32(inc).view(np.uint32)))
            hashes.append(sha(idx[:cnt]) + ":" + sha(val[:cnt].view(np.uint32)))
            if full:
                out[f"{name}/it{it}/idx"] = idx[:cnt].copy()
                out[f"{name}/it{it}/val"] = val[:cnt].copy()
        out[f"{name}/counts"] = np.array(counts, np.int64)
        out[f"{name}/t_bits"] = np.array(tbits, np.uint32)
        out[f"{name}/inc_bits"] = np.array(incbits, np.uint32)
        meta.append({"name": name, "n": n, "k": k, "dist": dist, "param": param, "iters": iters, "full": full,
                     "seed_bucket": 17, "key": "5@weight" if kind == "tv16" else "ptr", "hashes": hashes})
        (ref.tv16_free if kind == "tv16" else ref.tv_free)(h)
    return meta


def gen_topk(ref, out):
    meta = []
    for (name, n, k, dist, param) in TOPK_CASES:
        src = synth(n, seed_for(19, 0), dist, param)
        cnt, idx, val = ref.topk_compress(src, k)
        out[f"{name}/idx"] = idx.copy()
        out[f"{name}/val"] = val.copy()
        meta.append({"name": name, "n": n, "k": k, "dist": dist, "param": param, "seed_bucket": 19, "count": cnt})
    return meta


def gen_sgd(out):
    lib = C.CDLL(os.path.join(os.path.dirname(REF_SO), "libstg_ref_sgd.so"))
    f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
    u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
    lib.ref_sgd_new.restype = C.c_void_p
    lib.ref_sgd_new.argtypes = [C.c_float] * 4 + [C.c_int, C.c_int]
    lib.ref_sgd_apply.argtypes = [C.c_void_p, C.c_char_p, f32p, C.c_uint32, f32p, u32p, C.c_uint32]
    lib.ref_sgd_momentum.restype = C.c_int
    lib.ref_sgd_momentum.argtypes = [C.c_void_p, C.c_char_p, f32p, C.c_uint32]
    lib.ref_sgd_free.argtypes = [C.c_void_p]
    ref = Reference()
    meta = []
    for (name, n, k, lr, mom, damp, wd, nest, steps) in SGD_CASES:
        o = lib.ref_sgd_new(lr, mom, damp, wd, int(nest), 0)
        h = ref.tv16_new()
        param = synth(n, seed_for(23, 99), D1) * np.float32(1000.0)
        for s in range(steps):
            g = synth(n, seed_for(23, s), D1)
            cnt, idx, val = ref.tv16_compress(h, "p", g, k)
            lib.ref_sgd_apply(o, b"p", param, n, np.ascontiguousarray(val[:cnt]), np.ascontiguousarray(idx[:cnt]), cnt)
        mbuf = np.zeros(n, np.float32)
        has_m = lib.ref_sgd_momentum(o, b"p", mbuf, n) == 0
        out[f"{name}/param"] = param
        if has_m:
            out[f"{name}/momentum"] = mbuf
        meta.append({"name": name, "n": n, "k": k, "lr": lr, "momentum": mom, "dampening": damp,
                     "weight_decay": wd, "nesterov": nest, "steps": steps, "seed_bucket": 23,
                     "param_init": "synth(n, seed_for(23, 99), D1) * 1000", "grad_codec": "thresholdv16"})
        lib.ref_sgd_free(o)
        ref.tv16_free(h)
    return meta


def main():
    build(ref=True)
    ref = Reference()
    gxx = subprocess.run(["g++", "--version"], capture_output=True, text=True).stdout.splitlines()[0]
    manifest = {"producer": "reference backend/src/compress + optim/sgd.cpp compiled in place (oracle/Makefile)",
                "flags": "-std=c++17 -g -O3 -march=broadwell", "compiler": gxx, "host": platform.machine(),
                "generator": "stellatrain_amd/synth.py (splitmix64 Irwin-Hall, SURVEY 8(c))"}
    out: dict[str, np.ndarray] = {}
    manifest["tv16"] = gen_codec(ref, TV16_CASES, "tv16", out)
    manifest["tv"] = gen_codec(ref, TV_CASES, "tv", out)
    manifest["topk"] = gen_topk(ref, out)
    manifest["sgd"] = gen_sgd(out)
    np.savez_compressed(os.path.join(HERE, "golden.npz"), **out)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("wrote", len(out), "arrays;", os.path.getsize(os.path.join(HERE, "golden.npz")) >> 10, "KiB")


if __name__ == "__main__":
    main()
