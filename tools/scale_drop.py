#!/usr/bin/env python3
"""The regime-B fill after a drop of the gradient scale (DESIGN.md section 4,
the crew): a key converges on D1 data, then its gradients drop by a factor
(every line sum falls below the window under the threshold, so the fill
cannot take its pops from the scan's window list) and stay there for a few
calls while the AIMD threshold decays 1 % per call.

Every input is made and uploaded first; the calls then run back to back on
one stream, each bracketed by HIP events and preceded by a few copies that
keep the clocks up, each call's stream copied aside on the device.  Then
each call is compared with the oracle (test infrastructure, the check only).
Prints, per call, the device time, the count, and whether the whole stream
matches.

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
    steady = 8
    o = Oracle()
    comp = ThresholdvCompressor16()
    base = [o.synth(n, 9100 + c) for c in range(steady + drop)]
    junk_a = torch.empty(n, dtype=torch.float32, device=dev)
    junk_b = torch.empty_like(junk_a)
    st = torch.cuda.current_stream(dev)
    for fi, f in enumerate(factors):
        key = f"sd{fi}@weight"
        scales = [np.float32(1.0) if c < steady else np.float32(1.0 / f) for c in range(steady + drop)]
        srcs = [b * s for b, s in zip(base, scales)]
        dsrc = [torch.from_numpy(s).to(dev) for s in srcs]
        cnt = torch.zeros(len(srcs), dtype=torch.int64, device=dev)
        outi = torch.zeros((len(srcs), k), dtype=torch.int32, device=dev)
        outv = torch.zeros((len(srcs), k), dtype=torch.float32, device=dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in srcs]
        torch.cuda.synchronize()
        for c, d in enumerate(dsrc):
            for _ in range(4):  # keep the clocks up
                junk_b.copy_(junk_a)
            ev[c][0].record(st)
            cdev = comp.compress_async(key, d, k, outi[c], outv[c])
            ev[c][1].record(st)
            cnt[c] = cdev
        torch.cuda.synchronize()
        counts = cnt.cpu().numpy()
        hi, hv = outi.cpu().numpy().view(np.uint32), outv.cpu().numpy()
        ho = o.tv16_new()
        for c, src in enumerate(srcs):
            co, io, vo = o.tv16_compress(ho, key, src, k)
            ok = int(counts[c]) == co
            if ok:
                try:
                    assert_same_stream(hi[c], hv[c], io, vo, co)
                except AssertionError:
                    ok = False
            print(json.dumps({"drop": f, "call": c, "scale": float(scales[c]),
                              "us": round(ev[c][0].elapsed_time(ev[c][1]) * 1e3, 1), "count": int(counts[c]),
                              "stream_ok": ok}), flush=True)
        o.tv16_free(ho)
        del dsrc, outi, outv
    comp.check_device()


if __name__ == "__main__":
    main()
