"""kompressor_amd -- MI355X-native drop-in for Kompressor's lossless image / volume codec.

``import kompressor_amd as kom`` exposes the reference's API (``src/kompressor/__init__.py:24-26``):
``kom.image`` and ``kom.volume`` with ``encode`` / ``decode`` / ``encode_chunks`` /
``decode_chunks``, the geometry primitives, the residual coders and the losses, plus
``kom.predictors`` (built-in predictors the fused HIP kernels recognise), ``kom.packing``
(entropy-coded payloads of coded arrays: block-adaptive Rice / bit-planes) and ``kom.container``
(self-describing compressed files).  All arithmetic runs
in ``libkompressor_hip.so`` (hand-written gfx950 kernels behind the C-ABI in
``include/kompressor_hip.h``); there is no CPU fallback.
"""

from . import _lib  # noqa: F401  (fails loudly if libkompressor_hip.so is missing)
from . import image, volume, predictors, utils, tiles, shard, slabs, stream, packing, container, graphs  # noqa: F401
from .predictors import MeanPredictor, LinearPredictor  # noqa: F401
from ._device import release_pinned  # noqa: F401

VERSION = 'v1.0a'
