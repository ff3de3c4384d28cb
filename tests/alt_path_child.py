"""Child process of tests/test_gpu_alt_paths.py (not a test module).

Runs the codecs' opt-in launch shapes, selected by environment variables the
parent sets (read once per process): STG_TK2_FIN=1, Top-k's finish inside the
stream launch (topk1.hip tk2_finish); STG_TV_PASS=0, threshold-v's chunk
launches (tv.hip tv_chunk + tv_fold).  Every call's output is checked
against the oracle; prints one JSON line with the calls checked and the Top-k
debug words (38 band hits, 39 select calls, 49 calls finished in the stream
launch, 57 tk_one workgroups that ran anyway).
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def topk(dev, o, out):
    import torch
    from parity import assert_same_stream, assert_topk_values
    from stellatrain_amd import TopkCompressor
    from stellatrain_amd._capi import check, lib
    from stellatrain_amd.synth import D1, seed_for, synth
    calls = 0
    words = {}
    for bug_compat in (False, True):
        comp = TopkCompressor(exact=not bug_compat)
        # ragged n, a jump (band miss) and back; two keys interleaved
        for n, k in (((1 << 21) + 17, 20971), (1 << 24, 167772)):
            idx = torch.zeros(k, dtype=torch.int32, device=dev)
            val = torch.zeros(k, dtype=torch.float32, device=dev)
            for c, sc in enumerate([1, 1, 1, 10, 10, 1, 1]):
                for key in ("a", "b"):
                    x = synth(n, seed_for(910 + (key == "b"), c), D1) * np.float32(sc)
                    co, io, vo = o.topk_compress(x, k, idx_offset=0 if bug_compat else 5, bug_compat=bug_compat)
                    try:
                        cg = comp.compress(key, torch.from_numpy(x).to(dev), k, idx, val, 0 if bug_compat else 5)
                    except Exception:
                        w = (C.c_uint32 * 64)()
                        check(lib().stg_codec_debug_words(comp._h, C.c_void_p(torch.cuda.current_stream().cuda_stream),
                                                          w, 64))
                        print(json.dumps({"failed_call": [bug_compat, n, k, c, key], "words": list(w)}), flush=True)
                        raise
                    assert cg == co, (cg, co)
                    if bug_compat:
                        assert_topk_values(val.cpu().numpy(), vo)
                    else:
                        assert_same_stream(idx.cpu().numpy().view(np.uint32), val.cpu().numpy(), io, vo, k)
                    calls += 1
        comp.check_device()
        w = (C.c_uint32 * 64)()
        check(lib().stg_codec_debug_words(comp._h, C.c_void_p(torch.cuda.current_stream().cuda_stream), w, 64))
        words["shipped" if bug_compat else "exact"] = [w[38], w[39], w[49], w[57]]
    out["topk_calls"] = calls
    out["topk_words"] = words


def thresholdv(dev, o, out):
    import torch
    from parity import assert_same_stream
    from stellatrain_amd import ThresholdvCompressor
    from stellatrain_amd.synth import D1, D2, seed_for, synth
    calls = 0
    # ragged tails, a dense case (most chunk lists overflow: the re-read), a
    # bucket of one partial chunk
    for n, k, dist in ((100013, 100, D1), (1 << 20, 1048, D2), ((1 << 22) + 3, 1 << 21, D1), (5000, 4999, D1),
                       ((1 << 24) + 5, 16777, D1)):
        comp = ThresholdvCompressor()
        ho = o.tv_new()
        d = torch.empty(n, dtype=torch.float32, device=dev)
        for it in range(5):
            x = synth(n, seed_for(920, it), dist)
            co, io, vo = o.tv_compress(ho, 1, x, k)
            d.copy_(torch.from_numpy(x))
            idx = torch.zeros(k, dtype=torch.int32, device=dev)
            val = torch.zeros(k, dtype=torch.float32, device=dev)
            assert comp.compress("ignored", d, k, idx, val) == co
            assert_same_stream(idx.cpu().numpy().view(np.uint32), val.cpu().numpy(), io, vo, co)
            assert np.float32(comp.state("", key_ptr=d.data_ptr())[0]) == np.float32(o.tv_state(ho, 1))
            calls += 1
        comp.check_device()
    out["tv_calls"] = calls


def main():
    import torch
    from oracle.oracle import Oracle
    dev = torch.device("cuda", 0)
    o = Oracle()
    out = {}
    if os.environ.get("STG_TK2_FIN") == "1":
        topk(dev, o, out)
    if os.environ.get("STG_TV_PASS") == "0":
        thresholdv(dev, o, out)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
