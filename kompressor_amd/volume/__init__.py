"""``kompressor_amd.volume`` -- the 3D volume API, same names as ``kompressor.volume`` (volume/__init__.py:24-47)."""

from ..utils import \
    encode_values_raw, decode_values_raw, \
    encode_values_uint8, decode_values_uint8, \
    encode_values_uint16, decode_values_uint16, \
    encode_values_uint32, decode_values_uint32, \
    encode_categorical, decode_categorical  # noqa: F401

from .utils import \
    targets_from_highres, lowres_from_highres, \
    maps_from_predictions, maps_from_highres, \
    highres_from_lowres_and_maps, \
    features_from_lowres, pad_neighborhood  # noqa: F401

from .losses import \
    mean_squared_error, mean_abs_error, \
    mean_charbonnier_error, mean_total_variation  # noqa: F401

from .encode_decode import encode, decode, encode_pyramid, decode_pyramid  # noqa: F401
from .encode_decode_chunk import encode_chunks, decode_chunks  # noqa: F401
from . import utils, losses  # noqa: F401
