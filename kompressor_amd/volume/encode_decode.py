"""Whole-array encode / decode -- ``src/kompressor/volume/encode_decode.py`` of the reference.

With a built-in predictor (``kompressor_amd.predictors``) and a built-in coder whose modulus
matches the sample dtype, each call is ONE fused HIP kernel (libkompressor_hip.so); with any
other ``predictions_fn`` / coder it follows the reference's step sequence, each step a HIP
primitive, calling the user's functions exactly where the reference does.
"""

from .. import _nd

_N = 3


def encode(predictions_fn, encode_fn, highres, padding=0):
    """volume/encode_decode.py:30-56 -- returns ``(lowres, (maps, dims))``."""
    return _nd.encode(predictions_fn, encode_fn, highres, padding, _N)


def decode(predictions_fn, decode_fn, lowres, encoded, padding=0):
    """volume/encode_decode.py:59-85 -- returns the losslessly reconstructed highres."""
    return _nd.decode(predictions_fn, decode_fn, lowres, encoded, padding, _N)


def encode_pyramid(predictions_fn, encode_fn, highres, levels, padding=0):
    """Multi-level pyramid (build extension): ``encode`` applied ``levels``
    times, each on the previous lowres.  Returns ``(lowres, [(maps, dims), ...])``, finest first."""
    return _nd.encode_pyramid(predictions_fn, encode_fn, highres, levels, padding, _N)


def decode_pyramid(predictions_fn, decode_fn, lowres, encoded, padding=0):
    """Inverse of :func:`encode_pyramid`."""
    return _nd.decode_pyramid(predictions_fn, decode_fn, lowres, encoded, padding, _N)
