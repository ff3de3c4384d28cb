#!/usr/bin/env python3
"""Top-k band hits on the bench_configs C2 workload (64 MiB, k = 1 %, 9
rotating buffers of one key): debug words 38 (calls resolved in the band), 39
(calls that took the select's way), 49 (calls finished inside the stream
launch), per mode, after `calls` calls."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import torch
    from bench_configs import bufs_for
    from stellatrain_amd import TopkCompressor, merge_numel
    from stellatrain_amd._capi import check, lib
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n = 64 * (1 << 20) // 4
    k = merge_numel(n, 0.99)
    nbuf = 9
    bufs = bufs_for(torch, lib(), dev, n, nbuf, st.cuda_stream, 100)
    idx = torch.zeros(k, dtype=torch.int32, device=dev)
    val = torch.zeros(k, dtype=torch.float32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    keys = int(sys.argv[2]) if len(sys.argv) > 2 else 1  # bench_configs' C2 rows: 9 (a key per buffer)
    for exact in (False, True):
        comp = TopkCompressor(exact=exact)
        for i in range(calls):
            comp.compress_raw(f"{i % keys}@weight".encode(), bufs[i % nbuf].data_ptr(), n, k, idx.data_ptr(), k, val.data_ptr(),
                              cnt.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        w = (C.c_uint32 * 64)()
        check(lib().stg_codec_debug_words(comp._h, C.c_void_p(st.cuda_stream), w, 64))
        print({"exact": exact, "calls": calls, "keys": keys, "hits": w[38], "selects": w[39], "in_stream": w[49],
               "done_units": w[56], "tk_one_runs": w[57], "fin_miss": w[58], "fin_timeout": w[59]}, flush=True)
        comp.check_device()


if __name__ == "__main__":
    main()
