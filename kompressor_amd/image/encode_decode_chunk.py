"""Chunked encode / decode -- ``src/kompressor/image/encode_decode_chunk.py`` of the reference.

Windows come from ``yield_chunks`` (utils.py:114-155) and ``progress_fn`` receives the list of
chunks, as in the reference.  Results equal the whole-array calls.  On the fused path each chunk
is one region-restricted kernel launch.
"""

from .. import _nd

_N = 2


def encode_chunks(predictions_fn, encode_fn, highres, chunk=32, padding=0, progress_fn=None):
    """image/encode_decode_chunk.py:33-53."""
    return _nd.encode_chunks(predictions_fn, encode_fn, highres, chunk, padding, progress_fn, _N)


def decode_chunks(predictions_fn, decode_fn, lowres, encoded, chunk=32, padding=0, progress_fn=None):
    """image/encode_decode_chunk.py:56-74."""
    return _nd.decode_chunks(predictions_fn, decode_fn, lowres, encoded, chunk, padding, progress_fn, _N)


def process_chunks(predictions_fn, code_fn, lowres, reference_maps, chunk, padding, progress_fn):
    """image/encode_decode_chunk.py:77-115 (generic path, device tensors in and out)."""
    return _nd.d_process_chunks(predictions_fn, code_fn, lowres, reference_maps, chunk, padding, progress_fn, _N)
