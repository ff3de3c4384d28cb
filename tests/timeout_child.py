"""Child process of tests/test_gpu_failure_path.py (not a test module).

With STG_DEBUG_TK_WITHHOLD=1 set by the parent (read once per process),
Top-k's emission unit 0 never publishes its counts: every later unit's
look-back (topk1.hip emit_unit, in the stream launch's finish and again in
tk_one's) polls until its bound runs out and gives up.  The
failure has to surface end to end: the sticky failure word carries
FAIL_SPIN_TIMEOUT, the launch's count is poisoned (0xffffffff), the
synchronous compress() raises, and so does check_device().  Prints one JSON
line.
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from stellatrain_amd import CodecError, TopkCompressor
    from stellatrain_amd.synth import seed_for, synth
    dev = torch.device("cuda", 0)
    n, k = 1 << 22, 4194
    src = torch.from_numpy(synth(n, seed_for(77, 0))).to(dev)
    idx = torch.zeros(k, dtype=torch.int32, device=dev)
    val = torch.zeros(k, dtype=torch.float32, device=dev)
    comp = TopkCompressor(exact=True)
    out = {}
    comp.compress("w", src, k, idx, val)  # a key's first call: the select's way, which seeds the hint
    torch.cuda.synchronize()
    cnt = comp.compress_async("w", src, k, idx, val)
    torch.cuda.synchronize()
    out["count"] = int(cnt.item()) & 0xffffffff
    try:
        comp.check_device()
        out["check"] = "ok"
    except CodecError as e:
        out["check"] = str(e)
    try:
        comp.compress("w", src, k, idx, val)
        out["compress"] = "ok"
    except CodecError as e:
        out["compress"] = str(e)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
