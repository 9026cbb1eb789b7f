"""Image geometry primitives -- ``src/kompressor/image/utils.py`` of the reference, on the HIP
engine.  Arrays are channels-last ``[B, H, W, C...]``; numpy in -> numpy out, torch -> torch.
"""

from .. import _nd
from .._nd import yield_chunks, validate_padding  # noqa: F401  (re-exported like the reference)

_N = 2


def targets_from_highres(highres):
    """image/utils.py:37-49 -- the 5 per-cell training targets ``[B, cells..., 5, C...]``."""
    return _nd.wrap1(_nd.d_targets_from_highres)(highres, _N)


def lowres_from_highres(highres):
    """image/utils.py:52-55 -- skip sampling ``x[:, ::2, ::2]``."""
    return _nd.wrap1(_nd.d_lowres_from_highres)(highres, _N)


def maps_from_predictions(predictions):
    """image/utils.py:58-86 -- float32 aggregation of the 5 per-cell predictions onto 3 maps."""
    return _nd.wrap1(_nd.d_maps_from_predictions)(predictions, _N)


def maps_from_highres(highres):
    """image/utils.py:89-96 -- the 3 ground-truth maps (LR, UD, C)."""
    return _nd.wrap1(_nd.d_maps_from_highres)(highres, _N)


def highres_from_lowres_and_maps(lowres, maps):
    """image/utils.py:99-116 -- interleave lowres and the 3 maps."""
    return _nd.highres_from_lowres_and_maps(lowres, maps, _N)


def features_from_lowres(lowres, padding):
    """image/utils.py:120-129 -- ``[B, cells..., (2p+2)^2, C...]`` neighbourhood stack."""
    return _nd.wrap1(_nd.d_features_from_lowres)(lowres, padding, _N)


def pad_neighborhood(lowres, padding):
    """image/utils.py:132-137 -- symmetric pad of the spatial axes by ``padding``."""
    return _nd.wrap1(_nd.d_pad_neighborhood)(lowres, padding, _N)


def pad_highres(highres):
    """image/utils.py:145-156 -- reflect-pad even spatial dims by one; returns ``(padded, dims)``."""
    padded, dims = _nd.wrap1(lambda t, n: _nd.d_pad_highres(t, n)[0])(highres, _N), _nd.highres_dims(highres.shape, _N)
    return padded, dims


def pad_lowres(lowres, padding):
    """image/utils.py:159-163."""
    return _nd.wrap1(_nd.d_pad_lowres)(lowres, padding, _N)


def pad_map(inputs, padding):
    """image/utils.py:166-170."""
    return _nd.wrap1(lambda t, p, n: _nd.d_pad(t, (0,) * n, tuple(p), 0, n))(inputs, padding, _N)


def pad_maps(maps, padding):
    """image/utils.py:173-178."""
    return _nd.pad_maps(maps, padding, _N)


def trim(inputs, padding):
    """image/utils.py:181-185."""
    return _nd.wrap1(_nd.d_trim)(inputs, padding, _N)


def trim_maps(maps, padding):
    """image/utils.py:188-193."""
    return _nd.trim_maps(maps, padding, _N)


def validate_highres(highres):
    """image/utils.py:201-208."""
    return _nd.validate_highres_shape(highres.shape, _N)


def validate_lowres(lowres):
    """image/utils.py:211-218."""
    return _nd.validate_lowres_shape(lowres.shape, _N)


def validate_chunk(chunk):
    """image/utils.py:221-232."""
    return _nd.validate_chunk(chunk, _N)
