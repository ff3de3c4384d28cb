import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np, torch
from stellatrain_amd import ThresholdvCompressor16, merge_numel
from stellatrain_amd.synth import seed_for, synth
from oracle.oracle import Oracle
gpu = torch.device("cuda", 0)
o = Oracle()
n, N = 2097157, 9
k = merge_numel(n, 0.99)
for mode in ("ef", "plain"):
    comp = ThresholdvCompressor16(); ho = o.tv16_new()
    r_np = synth(n, seed_for(811, 0)) * np.float32(0.25)
    r = torch.from_numpy(r_np).to(gpu)
    for c in range(4):
        srcs = [synth(n, seed_for(812 + q, c)) for q in range(N)]
        x = srcs[0].copy()
        x = (x + r_np).astype(np.float32)
        for s_ in srcs[1:]: x = (x + s_).astype(np.float32)
        g = torch.from_numpy(x).to(gpu)
        i = torch.zeros(k, dtype=torch.int32, device=gpu); v = torch.zeros(k, dtype=torch.float32, device=gpu)
        if mode == "ef":
            cnt = comp.compress_batch_async([("g@w", g, k, i, v)], residuals=[r])
        else:
            cnt = comp.compress_async("g@w", g, k, i, v)
        torch.cuda.synchronize()
        co, io, vo = o.tv16_compress(ho, "g@w", x, k)
        gi = i.cpu().numpy().view(np.uint32)
        bad = np.nonzero(gi[:co] != io[:co])[0]
        print(mode, c, int(cnt[0].item()), co, "mismatch", bad.size, bad[:3].tolist(), bad[-3:].tolist() if bad.size else [], flush=True)
        if mode == "ef":  # the residual as the reference leaves it: src with the selected entries zeroed
            r_np = x.copy(); r_np[io[:co]] = 0
        comp.check_device()
