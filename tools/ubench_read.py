#!/usr/bin/env python3
"""Calibration: achievable HBM streaming rates on this MI355X for 64 MiB
buffers rotating through 1 GiB (torch copy / sum kernels), for comparison with
the codec's streaming pass."""
import json
import time

import torch

dev = torch.device("cuda:0")
n = 16 << 20
bufs = [torch.randn(n, device=dev) for _ in range(16)]
out = torch.empty(n, device=dev)
res = {}
for name, fn, bytes_per in [("copy", lambda x: out.copy_(x), 8 * n), ("sum", lambda x: x.sum(), 4 * n),
                            ("abs_max", lambda x: x.abs().max(), 8 * n)]:
    for i in range(16):
        fn(bufs[i])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 160
    for i in range(reps):
        fn(bufs[i % 16])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    res[name] = {"us": round(dt * 1e6, 2), "GBs": round(bytes_per / dt / 1e9, 1)}
print(json.dumps(res))
