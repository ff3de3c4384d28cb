"""GPU checks of the engine-facing call surface (not only the C-ABI underneath).

* ``CodecEngine.compress(name, tensor, ratio)`` is ``FasterDpEngine::compress``
  (engine/core.cpp:1210-1245): the ratio range check (:1212-1214), the API
  k = (long)((1 - ratio) * numel) (:1216), int32 indices (:1218), the k == 0
  early return (:1223-1225) and the narrowing to the returned count
  (:1236-1242), against the oracle.
* The compiled C++ shim (include/stg/compressor.h) driven by
  tests/cpp/shim_factory.cpp -- the reference factory of core.cpp:110-118 and
  the MERGE call of compress.cpp:141, unchanged -- run on the GPU box, its
  output file compared with the oracle (and with the reference build itself,
  oracle/_ref, when it travelled with the tree).
"""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

from parity import assert_same_pairs, assert_same_stream, bits
from stellatrain_amd.synth import D1, D2, seed_for, synth

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_engine_compress_api_thresholdv16(gpu, oracle):
    import torch
    from stellatrain_amd import CodecEngine, CodecError, api_numel
    eng = CodecEngine()  # thresholdv16 by default (core.cpp:23-26)
    n = 300007
    for bad in (-0.01, 1.5):
        with pytest.raises(CodecError, match=r"Ratio must be in range \[0, 1\]\."):
            eng.compress("x", torch.zeros(n, device=gpu), bad)
    i0, v0 = eng.compress("x", torch.zeros(n, device=gpu), 1.0)  # k == 0: empty, no codec call
    assert i0.numel() == 0 and v0.numel() == 0 and i0.dtype == torch.int32
    ho = oracle.tv16_new()
    for it in range(5):
        src = synth(n, seed_for(80, it), D1 if it % 2 else D2)
        k = api_numel(n, 0.99)
        co, io, vo = oracle.tv16_compress(ho, "api@weight", src, k)
        idx, val = eng.compress("api@weight", torch.from_numpy(src).to(gpu), 0.99)
        assert idx.dtype == torch.int32 and val.dtype == torch.float32
        assert idx.numel() == co == k  # thresholdv16 always fills dst_len
        assert_same_pairs(idx.cpu().numpy().view(np.uint32), val.cpu().numpy(), io, vo, co)
    oracle.tv16_free(ho)


def test_engine_compress_api_narrows_thresholdv(gpu, oracle):
    """threshold-v returns min(cnt, cap) (thresholdv.cpp:62-83): a call whose
    data shrank returns fewer than k pairs, and the API narrows both tensors."""
    import torch
    from stellatrain_amd import CodecEngine, api_numel
    eng = CodecEngine()
    eng.configure_compression("thresholdv")
    n = 200003
    k = api_numel(n, 0.999)
    buf = torch.empty(n, dtype=torch.float32, device=gpu)  # one buffer: pointer-keyed state
    ho = oracle.tv_new()
    narrowed = 0
    for it, scale in enumerate([1.0, 0.5, 0.5, 2.0, 1.0]):
        src = (synth(n, seed_for(81, it)) * np.float32(scale)).astype(np.float32)
        co, io, vo = oracle.tv_compress(ho, 1, src, k)
        buf.copy_(torch.from_numpy(src))
        idx, val = eng.compress("ignored", buf, 0.999)
        assert idx.numel() == val.numel() == co
        narrowed += co < k
        assert_same_stream(idx.cpu().numpy().view(np.uint32), val.cpu().numpy(), io, vo, co)
    assert narrowed
    oracle.tv_free(ho)


def test_engine_compress_api_host_tensor(gpu, oracle):
    """A CPU tensor takes the host path (stg_codec_compress_host), as the
    reference's compress() works on host memory."""
    import torch
    from stellatrain_amd import CodecEngine, api_numel
    eng = CodecEngine()
    n = 65536 + 9
    ho = oracle.tv16_new()
    for it in range(3):
        src = synth(n, seed_for(82, it))
        k = api_numel(n, 0.99)
        co, io, vo = oracle.tv16_compress(ho, "h", src, k)
        idx, val = eng.compress("h", torch.from_numpy(src), 0.99)
        assert idx.device.type == "cpu" and idx.numel() == co
        assert_same_pairs(idx.numpy().view(np.uint32), val.numpy(), io, vo, co)
    oracle.tv16_free(ho)


def _shim_binary():
    exe = os.path.join(ROOT, "tests", "cpp", "shim_factory")
    if not os.path.exists(exe):  # normally built by __graft_entry__.build()
        from stellatrain_amd.build import build_shim
        build_shim()
    return exe


def _read_shim(path, calls):
    data = open(path, "rb").read()
    out, p = [], 0
    for _ in range(calls):
        cnt = int(np.frombuffer(data, np.uint64, 1, p)[0])
        p += 8
        idx = np.frombuffer(data, np.uint32, cnt, p).copy()
        p += 4 * cnt
        val = np.frombuffer(data, np.float32, cnt, p).copy()
        p += 4 * cnt
        out.append((cnt, idx, val))
    assert p == len(data)
    return out


@pytest.mark.parametrize("method", ["thresholdv16", "thresholdv", "topk"])
def test_cpp_shim_binary_matches_oracle(gpu, oracle, method, tmp_path):
    """The engine-shaped boundary end to end: the reference factory and call
    site compiled against include/stg/compressor.h, running on the GPU."""
    n = 1 << 20
    k = oracle.merge_numel(n, 0.99)
    calls = 4
    src = synth(n, seed_for(83, 0))
    fin, fout = tmp_path / "in.f32", tmp_path / "out.bin"
    src.tofile(fin)
    r = subprocess.run([_shim_binary(), method, str(fin), str(k), str(fout), str(calls)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == {"thresholdv16": "Thresholdv16", "thresholdv": "Thresholdv", "topk": "Topk"}[method] + " ok"
    got = _read_shim(fout, calls)
    from oracle.oracle import Reference, reference_available
    refs = [oracle] + ([Reference()] if reference_available() and os.path.exists(
        os.path.join(ROOT, "oracle", "_ref", "libstg_ref.so")) else [])
    for chk in refs:
        if method == "thresholdv16":
            h = chk.tv16_new()
            exp = [chk.tv16_compress(h, "3@weight", src, k) for _ in range(calls)]
            chk.tv16_free(h)
        elif method == "thresholdv":
            h = chk.tv_new()
            # the shim's host path keys threshold-v by its (stable) src pointer
            exp = [chk.tv_compress(h, 1, src, k) for _ in range(calls)]
            chk.tv_free(h)
        else:
            exp = [chk.topk_compress(src, k) for _ in range(calls)]
        for (cg, ig, vg), (ce, ie, ve) in zip(got, exp):
            assert cg == ce
            if method == "topk":
                np.testing.assert_array_equal(ig, np.arange(k))
                from parity import assert_topk_values
                assert_topk_values(vg, ve[:ce])
            else:
                assert_same_pairs(ig, vg, ie, ve, ce)
                if method == "thresholdv":
                    assert_same_stream(ig, vg, ie, ve, ce)
    assert bits(got[0][2]).size == got[0][0]
