"""Child process of tests/test_gpu_coresidency.py (not a test module).

Issues thresholdv16 batches on S streams at once with STG_TV16_INFLIGHT set
by the parent (read once per process), optionally with a foreign GEMM loop
occupying CUs on another stream, and checks every bucket's stream against
the oracle and the device failure word.  Prints one JSON line.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    streams = int(sys.argv[1])
    gemm = int(sys.argv[2])
    import torch
    from oracle.oracle import Oracle
    from parity import assert_same_stream
    from stellatrain_amd import ThresholdvCompressor16, merge_numel
    from stellatrain_amd.synth import seed_for, synth
    dev = torch.device("cuda", 0)
    o = Oracle()
    ho = o.tv16_new()
    comp = ThresholdvCompressor16()
    n = (4 << 20) // 4 + 16 * 3  # 4 MiB + 3 lines: 9 chunks per bucket
    k = merge_numel(n, 0.99)
    per = 4  # buckets per batch
    keys = [f"s{s}b{j}" for s in range(streams) for j in range(per)]
    sts = [torch.cuda.Stream(dev) for _ in range(streams)]
    g_stream = torch.cuda.Stream(dev)
    a = torch.randn(8192, 8192, dtype=torch.bfloat16, device=dev)
    b = torch.randn(8192, 8192, dtype=torch.bfloat16, device=dev)
    checked = 0
    for it in range(4):
        srcs = [synth(n, seed_for(100 + i, it)) for i in range(len(keys))]
        dsrc = [torch.from_numpy(x).to(dev) for x in srcs]
        outs = [(torch.zeros(k, dtype=torch.int32, device=dev), torch.zeros(k, dtype=torch.float32, device=dev))
                for _ in keys]
        torch.cuda.synchronize()
        if gemm:  # CUs busy with somebody else's kernels while the codec runs
            with torch.cuda.stream(g_stream):
                for _ in range(gemm):
                    a = (a @ b) * 1e-3
        counts = []
        for s, st in enumerate(sts):
            ids = range(s * per, (s + 1) * per)
            with torch.cuda.stream(st):
                counts.append(comp.compress_batch_async([(keys[i], dsrc[i], k, outs[i][0], outs[i][1]) for i in ids],
                                                        stream=st.cuda_stream))
        torch.cuda.synchronize()
        for s in range(streams):
            for j, i in enumerate(range(s * per, (s + 1) * per)):
                co, io, vo = o.tv16_compress(ho, keys[i], srcs[i], k)
                assert int(counts[s][j].item()) == co, (it, i)
                assert_same_stream(outs[i][0].cpu().numpy().view(np.uint32), outs[i][1].cpu().numpy(), io, vo, co)
                checked += 1
    comp.check_device()
    print(json.dumps({"ok": True, "streams": streams, "gemm": gemm, "buckets_checked": checked,
                      "inflight": os.environ.get("STG_TV16_INFLIGHT")}), flush=True)


if __name__ == "__main__":
    main()
