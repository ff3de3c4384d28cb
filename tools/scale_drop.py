#!/usr/bin/env python3
"""The regime-B fill after a drop of the gradient scale (DESIGN.md section 4,
the crew): a key converges on D1 data, then its gradients drop by a factor
(every line sum falls below the window under the threshold, so the fill
cannot take its pops from the scan's window list) and stay there for a few
calls while the AIMD threshold decays 1 % per call.  Prints, per call, the
time of a lone compress() (HIP events around the call, which returns after
the count is read back; one call at a time), the count, and whether the
whole stream matches the oracle (test infrastructure, the check only).

    tools/scale_drop.py [calls after the drop] [drop factors, comma-separated]
"""
import json
import os
import sys

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
    drop = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    factors = [float(f) for f in sys.argv[2].split(",")] if len(sys.argv) > 2 else [100.0]
    o = Oracle()
    comp = ThresholdvCompressor16()
    idx = torch.zeros(k, dtype=torch.int32, device=dev)
    val = torch.zeros(k, dtype=torch.float32, device=dev)
    steady = 8
    for fi, f in enumerate(factors):
        ho = o.tv16_new()
        key = f"sd{fi}@weight"
        for c in range(steady + drop):
            scale = np.float32(1.0) if c < steady else np.float32(1.0 / f)
            src = o.synth(n, 9100 + c) * scale
            d = torch.from_numpy(src).to(dev)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            cg = comp.compress(key, d, k, idx, val)  # returns after the count is read back
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3
            co, io, vo = o.tv16_compress(ho, key, src, k)
            ok = cg == co
            if ok:
                try:
                    assert_same_stream(idx.cpu().numpy().view(np.uint32), val.cpu().numpy(), io, vo, co)
                except AssertionError:
                    ok = False
            print(json.dumps({"drop": f, "call": c, "scale": float(scale), "us": round(us, 1), "count": int(cg),
                              "stream_ok": ok}), flush=True)
        o.tv16_free(ho)
    comp.check_device()


if __name__ == "__main__":
    main()
