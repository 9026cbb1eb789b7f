"""Volume geometry primitives -- ``src/kompressor/volume/utils.py`` of the reference, on the HIP
engine.  Arrays are channels-last ``[B, D, H, W, C...]``; numpy in -> numpy out, torch -> torch.
"""

from .. import _nd
from .._nd import yield_chunks, validate_padding  # noqa: F401  (re-exported like the reference)

_N = 3


def targets_from_highres(highres):
    """volume/utils.py:37-74 -- the 19 per-cell training targets ``[B, cells..., 19, C...]``."""
    return _nd.wrap1(_nd.d_targets_from_highres)(highres, _N)


def lowres_from_highres(highres):
    """volume/utils.py:77-80 -- skip sampling ``x[:, ::2, ::2, ::2]``."""
    return _nd.wrap1(_nd.d_lowres_from_highres)(highres, _N)


def maps_from_predictions(predictions):
    """volume/utils.py:83-155 -- float32 aggregation of the 19 per-cell predictions onto 7 maps."""
    return _nd.wrap1(_nd.d_maps_from_predictions)(predictions, _N)


def maps_from_highres(highres):
    """volume/utils.py:158-171 -- the 7 ground-truth maps (LR, UD, FB, C, Z, Y, X)."""
    return _nd.wrap1(_nd.d_maps_from_highres)(highres, _N)


def highres_from_lowres_and_maps(lowres, maps):
    """volume/utils.py:174-195 -- interleave lowres and the 7 maps."""
    return _nd.highres_from_lowres_and_maps(lowres, maps, _N)


def features_from_lowres(lowres, padding):
    """volume/utils.py:199-210 -- ``[B, cells..., (2p+2)^3, C...]`` neighbourhood stack."""
    return _nd.wrap1(_nd.d_features_from_lowres)(lowres, padding, _N)


def pad_neighborhood(lowres, padding):
    """volume/utils.py:213-218 -- symmetric pad of the spatial axes by ``padding``."""
    return _nd.wrap1(_nd.d_pad_neighborhood)(lowres, padding, _N)


def pad_highres(highres):
    """volume/utils.py:226-237 -- reflect-pad even spatial dims by one; returns ``(padded, dims)``."""
    padded, dims = _nd.wrap1(lambda t, n: _nd.d_pad_highres(t, n)[0])(highres, _N), _nd.highres_dims(highres.shape, _N)
    return padded, dims


def pad_lowres(lowres, padding):
    """volume/utils.py:240-244."""
    return _nd.wrap1(_nd.d_pad_lowres)(lowres, padding, _N)


def pad_map(inputs, padding):
    """volume/utils.py:247-251."""
    return _nd.wrap1(lambda t, p, n: _nd.d_pad(t, (0,) * n, tuple(p), 0, n))(inputs, padding, _N)


def pad_maps(maps, padding):
    """volume/utils.py:254-260."""
    return _nd.pad_maps(maps, padding, _N)


def trim(inputs, padding):
    """volume/utils.py:263-267."""
    return _nd.wrap1(_nd.d_trim)(inputs, padding, _N)


def trim_maps(maps, padding):
    """volume/utils.py:270-276."""
    return _nd.trim_maps(maps, padding, _N)


def validate_highres(highres):
    """volume/utils.py:284-292."""
    return _nd.validate_highres_shape(highres.shape, _N)


def validate_lowres(lowres):
    """volume/utils.py:295-303."""
    return _nd.validate_lowres_shape(lowres.shape, _N)


def validate_chunk(chunk):
    """volume/utils.py:306-318."""
    return _nd.validate_chunk(chunk, _N)
