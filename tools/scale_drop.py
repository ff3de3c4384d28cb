#!/usr/bin/env python3
"""The regime-B fill's worst case at 64 MiB (DESIGN.md section 4 fill item 5):
a key converges on D1 data, then its gradients drop 100x (every line sum
falls below the window under the threshold), so the fill runs the literal
heap until the AIMD threshold decays back.  Prints, per call, the device time
of a lone compress() (HIP events, one call at a time), the count, and whether
the whole stream matches the oracle (test infrastructure, the check only)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    from oracle.oracle import Oracle
    from parity import assert_same_stream
    from stellatrain_amd import ThresholdvCompressor16, merge_numel
    dev = torch.device("cuda", 0)
    n = 16 << 20
    k = merge_numel(n, 0.99)
    o = Oracle()
    ho = o.tv16_new()
    comp = ThresholdvCompressor16()
    idx = torch.zeros(k, dtype=torch.int32, device=dev)
    val = torch.zeros(k, dtype=torch.float32, device=dev)
    steady, drop = 8, int(sys.argv[1]) if len(sys.argv) > 1 else 6
    for c in range(steady + drop):
        scale = np.float32(1.0) if c < steady else np.float32(0.01)
        src = o.synth(n, 9100 + c) * scale
        d = torch.from_numpy(src).to(dev)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        cg = comp.compress("sd@weight", d, k, idx, val)  # returns after the count is read back
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3
        co, io, vo = o.tv16_compress(ho, "sd@weight", src, k)
        ok = cg == co
        if ok:
            try:
                assert_same_stream(idx.cpu().numpy().view(np.uint32), val.cpu().numpy(), io, vo, co)
            except AssertionError:
                ok = False
        print(json.dumps({"call": c, "scale": float(scale), "us": round(us, 1), "count": int(cg), "stream_ok": ok}),
              flush=True)
    comp.check_device()
    o.tv16_free(ho)


if __name__ == "__main__":
    main()
