"""The intra-node gather-add fused into the codec's streaming pass
(stg_merge_gather_compress_device): ModuleCpuGather::run
(engine/modules/cpu_gather.cpp:59-87, add_arrays misc/array_util.h:12-52)
then ModuleCompress::run (engine/modules/compress.cpp:139-186) on one slice.

Checked against the same task as separate GPU calls (the adds in order, then
stg_merge_compress_batch_device / stg_codec_compress_device) on a second
codec handle, bit for bit: the stream, the count, grad[0] after the task, the
residual, and the key's threshold; and the stream against the oracle run on
the numpy sum in the reference's order.  A key's first call (the gather runs
as its own pass), steady calls (fused), ragged tails, N = 1, 2, 4 and 9, with
and without the residual."""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np
import pytest

from parity import assert_same_stream

pytestmark = pytest.mark.gpu


def _words(comp, stream):
    from stellatrain_amd._capi import check, lib
    w = (C.c_uint32 * 64)()
    check(lib().stg_codec_debug_words(comp._h, C.c_void_p(stream.cuda_stream), w, 64))
    return list(w)


def _np_gather(g, resid):
    acc = g[0].copy()
    if resid is not None:
        acc = (acc + resid).astype(np.float32)
    for x in g[1:]:
        acc = (acc + x).astype(np.float32)
    return acc


@pytest.mark.parametrize("n,N,with_resid", [((1 << 22) + 13, 2, True), ((1 << 22) + 13, 4, False),
                                            (1 << 20, 1, True), ((1 << 21) + 5, 9, True)])
def test_gather_fused_matches_separate(gpu, oracle, n, N, with_resid):
    import torch
    from stellatrain_amd import ThresholdvCompressor16, merge_numel
    from stellatrain_amd.synth import seed_for, synth
    k = merge_numel(n, 0.99)
    fused, sep = ThresholdvCompressor16(), ThresholdvCompressor16()
    ho = oracle.tv16_new()
    rng_resid = synth(n, seed_for(811, 0)) * np.float32(0.25) if with_resid else None
    r_f = torch.from_numpy(rng_resid).to(gpu) if with_resid else None
    r_s = r_f.clone() if with_resid else None
    r_np = rng_resid.copy() if with_resid else None
    try:
        for c in range(4):
            srcs = [synth(n, seed_for(812 + r, c)) for r in range(N)]
            g_f = [torch.from_numpy(x).to(gpu) for x in srcs]
            g_s = [t.clone() for t in g_f]
            i_f = torch.zeros(k, dtype=torch.int32, device=gpu)
            v_f = torch.zeros(k, dtype=torch.float32, device=gpu)
            i_s, v_s = torch.zeros_like(i_f), torch.zeros_like(v_f)
            cnt_f = fused.merge_gather_compress_async("g@w", g_f, k, i_f, v_f, residual=r_f)
            if with_resid:  # the gather-add as separate ops (each add correctly rounded, in order)
                g_s[0].add_(r_s)
            for t in g_s[1:]:
                g_s[0].add_(t)
            if with_resid:
                cnt_s = sep.compress_batch_async([("g@w", g_s[0], k, i_s, v_s)], residuals=[r_s])
            else:
                cnt_s = sep.compress_async("g@w", g_s[0], k, i_s, v_s)
            torch.cuda.synchronize()
            # each side against the oracle on the reference's sum first, so a
            # failure names the side that is wrong
            x = _np_gather(srcs, r_np)
            t_in = oracle.tv16_state(ho, "g@w")[0] if c else None
            co, io, vo = oracle.tv16_compress(ho, "g@w", x, k)
            t_out = oracle.tv16_state(ho, "g@w")[0]
            regime = "first call" if not c else ("B" if t_out < t_in else "A")  # (B decays t by 1 %)
            what = f"call {c} (n={n}, N={N}, resid={with_resid}, t_in={t_in}, oracle count {co}, regime {regime})"
            for side, cnt, ii, vv in (("fused", cnt_f, i_f, v_f), ("separate", cnt_s[0], i_s, v_s)):
                assert int(cnt.item()) == co, f"{side} count {int(cnt.item())} != {co}: {what}"
                assert_same_stream(ii.cpu().numpy().view(np.uint32), vv.cpu().numpy(), io, vo, co, f"{side} vs oracle, {what}")
            np.testing.assert_array_equal(g_f[0].cpu().numpy().view(np.uint32), g_s[0].cpu().numpy().view(np.uint32))
            if with_resid:
                np.testing.assert_array_equal(r_f.cpu().numpy().view(np.uint32), r_s.cpu().numpy().view(np.uint32))
            assert np.float32(fused.state("g@w")[0]) == np.float32(sep.state("g@w")[0]), what
            if with_resid:
                r_np = r_f.cpu().numpy().copy()
        fused.check_device()
        sep.check_device()
        # the in-scan finish's freshness check (tv16lf2.h): in production it never
        # has to send a call to the fill launch (every list entry carries its
        # call's tag); with STG_LF2_SKIP=5 the scan tags its lists wrongly and
        # every call with qualifying lines must go there, bit-exact all the same
        st = torch.cuda.current_stream()
        if os.environ.get("STG_LF2_SKIP") == "5":
            assert _words(fused, st)[31] > 0 and _words(sep, st)[31] > 0
        else:
            assert _words(fused, st)[31] == 0 and _words(sep, st)[31] == 0
    finally:
        oracle.tv16_free(ho)


@pytest.mark.skipif(os.environ.get("STG_LF2_SKIP") == "5", reason="already the wrong-tag run")
def test_gather_fused_wrong_tag_lists_fall_back(gpu):
    """The four cases above in a child process whose scans tag their lists with
    a wrong call tag (STG_LF2_SKIP=5, read once per process): the finish's
    freshness check must hand every call to the fill launch, and every stream
    must still match the oracle and the separate calls."""
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, STG_LF2_SKIP="5")
    r = subprocess.run([sys.executable, "-m", "pytest", os.path.join(here, "test_gpu_gather_fused.py"), "-q", "-m", "gpu",
                        "-k", "matches_separate", "-p", "no:cacheprovider"],
                       env=env, cwd=os.path.dirname(here), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
