#!/usr/bin/env python3
"""Generate tests/golden/golden_configs.npz + manifest_configs.json: the
REFERENCE's own outputs at every BASELINE.json config's full size.

Producer: oracle/_ref/libstg_ref.so / libstg_ref_sgd.so -- the reference's
backend/src/compress/{thresholdv16,thresholdv,topk}.cpp and optim/sgd.cpp
compiled in place from /root/reference (-g -O3 -march=broadwell,
backend/CMakeLists.txt:28-32) by oracle/Makefile.  Inputs are not stored: they
are regenerated bit-exactly from (n, seed, dist, scale) by the integer-only
generator (stellatrain_amd/synth.py == csrc/synth.hip == orc_synth_fill).

  C1  thresholdv16, n = 4,194,304, k = 41,943, 32 AIMD calls on one key
      (SURVEY 8(c)(ii)): full idx of calls 0-3, and for every call the count,
      the threshold bits, sha256 of the (idx, val) stream in order and of the
      pair set (sorted by idx).
  C2  top-k (shipped), n = 16,777,216, k = 167,772: count and sha256 of the
      sorted signed value bits (the nth_element partition order is free).
  C3  threshold-v, n = 67,108,864, k = cap = 67,108, 10 calls whose input scale
      varies (cnt > cap overflow and cnt < k both occur): counts, threshold
      bits, stream sha256; full idx of call 0.
  C4  the 1,024-bucket stream (shard.c4_sizes), 2 sweeps (the engine's iter%2
      buffers): per bucket and sweep the count, threshold bits, set sha256 and
      stream sha256 (the regime-B heap fill's pop order, thresholdv16.cpp:261-293).
  C5  64 MiB compress -> MERGE decompress (world 1) -> momentum SGD, 3 steps:
      sha256 of param and momentum after every step.

    python tests/golden/make_golden_configs.py [--only c1,c2,...]
"""
from __future__ import annotations

import argparse
import ctypes as C
import hashlib
import json
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.oracle import REF_SO, Oracle, Reference, build  # noqa: E402
from stellatrain_amd.engine import merge_numel  # noqa: E402
from stellatrain_amd.shard import ShardPlan, c4_sizes  # noqa: E402
from stellatrain_amd.synth import D1, seed_for  # noqa: E402

C1 = dict(n=4194304, k=41943, calls=32, bucket=101, key="c1@weight", full_calls=4)
C2 = dict(n=16777216, k=167772, bucket=102)
C3 = dict(n=67108864, k=67108, bucket=103, scales=[1.0, 1.0, 0.9, 1.1, 1.0, 0.95, 1.05, 1.0, 1.2, 0.8])
C4 = dict(sweeps=2)
C5 = dict(n=16777216, k=167772, steps=3, bucket=105, param_bucket=106, lr=0.1, momentum=0.9)


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def stream_sha(idx, val, cnt) -> str:
    return sha(idx[:cnt]) + ":" + sha(np.ascontiguousarray(val[:cnt], np.float32).view(np.uint32))


def set_sha(idx, val, cnt) -> str:
    i = np.asarray(idx[:cnt], np.uint32)
    o = np.argsort(i, kind="stable")
    return stream_sha(i[o], np.asarray(val[:cnt], np.float32)[o], cnt)


def tbits(t) -> int:
    return int(np.float32(t).view(np.uint32))


def gen(o, n, seed, scale=1.0):
    x = o.synth(n, seed, D1)
    if scale != 1.0:
        x = (x * np.float32(scale)).astype(np.float32)
    return x


def c1(ref, o, out):
    h = ref.tv16_new()
    rows = []
    for it in range(C1["calls"]):
        src = gen(o, C1["n"], seed_for(C1["bucket"], it))
        cnt, idx, val = ref.tv16_compress(h, C1["key"], src, C1["k"])
        t, inc = ref.tv16_state(h, C1["key"])
        rows.append({"count": cnt, "t_bits": tbits(t), "inc_bits": tbits(inc), "stream": stream_sha(idx, val, cnt),
                     "set": set_sha(idx, val, cnt)})
        if it < C1["full_calls"]:
            out[f"c1/it{it}/idx"] = idx[:cnt].copy()
    ref.tv16_free(h)
    return dict(C1, rows=rows)


def c2(ref, o):
    src = gen(o, C2["n"], seed_for(C2["bucket"], 0))
    cnt, idx, val = ref.topk_compress(src, C2["k"])
    v = np.asarray(val[:cnt], np.float32)
    cut = float(np.abs(v).min())
    above = np.sort(v[np.abs(v) > cut].view(np.uint32))
    return dict(C2, count=cnt, cut_bits=tbits(cut), above_sorted_sha=sha(above), at_cut=int((np.abs(v) == cut).sum()),
                idx_is_arange=bool(np.array_equal(idx[:cnt], np.arange(cnt))))


def c3(ref, o, out):
    h = ref.tv_new()
    rows = []
    for it, sc in enumerate(C3["scales"]):
        src = gen(o, C3["n"], seed_for(C3["bucket"], it), sc)
        cnt, idx, val = ref.tv_compress(h, 1, src, C3["k"])
        t = ref.tv_state(h, 1)
        # cnt is min(count, cap): the uncapped count is not returned; record
        # whether the scan overflowed from the threshold move (thresholdv.cpp:72-80)
        rows.append({"count": cnt, "t_bits": tbits(t), "stream": stream_sha(idx, val, cnt)})
        if it == 0:
            out["c3/it0/idx"] = idx[:cnt].copy()
    ref.tv_free(h)
    return dict(C3, rows=rows)


def c4(ref, o):
    sizes = c4_sizes()
    plan = ShardPlan(sizes, 1)
    h = ref.tv16_new()
    rows = []
    t0 = time.time()
    for sw in range(C4["sweeps"]):
        for b, n in enumerate(sizes):
            k = merge_numel(n, 0.99)
            src = gen(o, n, seed_for(b, sw))
            cnt, idx, val = ref.tv16_compress(h, plan.key(b), src, k)
            t, _ = ref.tv16_state(h, plan.key(b))
            rows.append([sw, b, cnt, tbits(t), set_sha(idx, val, cnt), stream_sha(idx, val, cnt)])
        print(f"  c4 sweep {sw} done ({time.time() - t0:.0f} s)", flush=True)
    ref.tv16_free(h)
    return dict(C4, count=len(sizes), sizes_sha=sha(np.array(sizes, np.int64)), rows=rows)


def c5(ref, o):
    lib = C.CDLL(os.path.join(os.path.dirname(REF_SO), "libstg_ref_sgd.so"))
    f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
    u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
    lib.ref_sgd_new.restype = C.c_void_p
    lib.ref_sgd_new.argtypes = [C.c_float] * 4 + [C.c_int, C.c_int]
    lib.ref_sgd_apply.argtypes = [C.c_void_p, C.c_char_p, f32p, C.c_uint32, f32p, u32p, C.c_uint32]
    lib.ref_sgd_momentum.restype = C.c_int
    lib.ref_sgd_momentum.argtypes = [C.c_void_p, C.c_char_p, f32p, C.c_uint32]
    lib.ref_sgd_free.argtypes = [C.c_void_p]
    n, k = C5["n"], C5["k"]
    sgd = lib.ref_sgd_new(C5["lr"], C5["momentum"], 0.0, 0.0, 0, 0)
    h = ref.tv16_new()
    param = gen(o, n, seed_for(C5["param_bucket"], 0))
    rows = []
    for s in range(C5["steps"]):
        g = gen(o, n, seed_for(C5["bucket"], s))
        cnt, idx, val = ref.tv16_compress(h, "c5@weight", g, k)
        # MERGE decompress, world 1 (cpu_optimize.cpp:40-72): zeros + index_put_,
        # merged = 0 + tmp, / 1.0, gathered at the unique indices
        tmp = np.zeros(n, np.float32)
        tmp[idx[:cnt]] = val[:cnt]
        merged = (np.zeros(n, np.float32) + tmp) / np.float32(1.0)
        uidx = np.unique(idx[:cnt]).astype(np.uint32)
        uval = np.ascontiguousarray(merged[uidx])
        lib.ref_sgd_apply(sgd, b"c5@weight", param, n, uval, uidx, uidx.size)
        mom = np.zeros(n, np.float32)
        assert lib.ref_sgd_momentum(sgd, b"c5@weight", mom, n) == 0
        rows.append({"count": cnt, "merged": int(uidx.size), "param": sha(param.view(np.uint32)),
                     "momentum": sha(mom.view(np.uint32))})
    lib.ref_sgd_free(sgd)
    ref.tv16_free(h)
    return dict(C5, rows=rows)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="c1,c2,c3,c4,c5")
    only = set(ap.parse_args().only.split(","))
    build(ref=True)
    ref, o = Reference(), Oracle()
    path_m = os.path.join(HERE, "manifest_configs.json")
    path_a = os.path.join(HERE, "golden_configs.npz")
    man = json.load(open(path_m)) if os.path.exists(path_m) else {}
    arrs = dict(np.load(path_a)) if os.path.exists(path_a) else {}
    gxx = subprocess.run(["g++", "--version"], capture_output=True, text=True).stdout.splitlines()[0]
    man.update({"producer": "reference backend/src/compress + optim/sgd.cpp compiled in place (oracle/Makefile)",
                "flags": "-std=c++17 -g -O3 -march=broadwell", "compiler": gxx,
                "generator": "orc_synth_fill == stellatrain_amd/synth.py (splitmix64 Irwin-Hall D1), seed_for(bucket, "
                             "call); scaled inputs are (synth * float32(scale)) in float32"})
    for name, fn in (("c1", lambda: c1(ref, o, arrs)), ("c2", lambda: c2(ref, o)), ("c3", lambda: c3(ref, o, arrs)),
                     ("c4", lambda: c4(ref, o)), ("c5", lambda: c5(ref, o))):
        if name in only:
            t0 = time.time()
            man[name] = fn()
            print(name, f"{time.time() - t0:.1f} s", flush=True)
    np.savez_compressed(path_a, **arrs)
    with open(path_m, "w") as f:
        json.dump(man, f, indent=1)
    print("wrote", path_a, os.path.getsize(path_a) >> 10, "KiB")


if __name__ == "__main__":
    main()
