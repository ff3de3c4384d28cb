"""stellatrain_amd -- MI355X-native gradient-sparsification codec.

A drop-in for StellaTrain's CPU compress path (backend/src/compress): the
thresholdv16 / threshold-v / Top-k codecs, the MERGE decompress and the
sparse SGD apply, as hand-written HIP kernels for gfx950 behind the C-ABI in
include/stg/codec.h.  See DESIGN.md.
"""
from ._capi import CodecError, lib  # noqa: F401
from .compressor import (Compressor, ThresholdvCompressor, ThresholdvCompressor16, TopkCompressor,  # noqa: F401
                         make_compressor)
from .engine import (CodecEngine, SparseAdam, SparseSGD, api_numel, merge_numel, owner_of,  # noqa: F401
                     gather_add, gather_slice, scatter_merge, wire_decode, wire_encode, wire_encode_batch,
                     wire_flag)

__version__ = "0.1.0"
