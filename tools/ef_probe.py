"""Which heap-fill path the MERGE+EF benchmark's calls take (diagnostic)."""
import ctypes as C, os, sys, time, json
sys.path.insert(0, os.getcwd())
import torch
from stellatrain_amd import ThresholdvCompressor16, merge_numel
from stellatrain_amd._capi import check, lib
from stellatrain_amd.synth import seed_for
dev = torch.device("cuda", 0); st = torch.cuda.current_stream(dev)
n = 16 << 20; k = merge_numel(n, 0.99); nb = 16
grads = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(nb)]
res = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(nb)]
idx = [torch.zeros(k, dtype=torch.int32, device=dev) for _ in range(nb)]
val = [torch.zeros(k, dtype=torch.float32, device=dev) for _ in range(nb)]
comp = ThresholdvCompressor16()
counts = torch.zeros(nb, dtype=torch.int32, device=dev)
def words():
    w = (C.c_uint32 * 64)()
    check(lib().stg_codec_debug_words(comp._h, C.c_void_p(st.cuda_stream), w, 64))
    return list(w)[56:64]
for rep, seeds in enumerate([range(4), range(12)]):
    for s in seeds:
        for h in range(2):
            sl = range(8 * h, 8 * h + 8)
            for j in sl:
                check(lib().stg_synth_fill_device(C.c_void_p(grads[j].data_ptr()), n, seed_for(500 + j, s), 0, 0, C.c_void_p(st.cuda_stream)))
            comp.compress_batch_async([(f"{j}@w", grads[j], k, idx[j], val[j]) for j in sl], counts=counts[8 * h:],
                                      residuals=[res[j] for j in sl])
        torch.cuda.synchronize()
        ws = words()
        print(json.dumps({"rep": rep, "seed": s, "paths": ws[:4], "why_literal(nowin,N,W,covered)": ws[4:],
                          "t": [round(comp.state(f"{j}@w")[0], 9) for j in (0, 8)]}), flush=True)
