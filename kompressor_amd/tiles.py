"""Split one volume (image) into a batch of independent tiles and reassemble it, on the GPU.

BASELINE configs C3/C4 code ONE 512^3 volume as 512 tiles of 64^3: the
tiles become the leading batch axis that every reference primitive is parallel over
(``volume/utils.py:80,161-169``), so each tile gets its own even-dim padding and predictor
boundary handling exactly as if it were a separate array.  Tile order is z-major
(``(tz * nty + ty) * ntx + tx``).  The permutation runs in ``kmp_tiles`` (kmp_tiles.hip).
"""

from . import _device as dev
from . import _lib
from ._lib import check, lib


def _split_shape(shape, nsp):
    sp = tuple(int(s) for s in shape[:nsp])
    ch = tuple(int(s) for s in shape[nsp:])
    return sp, ch


def volume_to_tiles(volume, tile, ndim=3):
    """``volume`` [D, H, W, C...] (image: [H, W, C...]) -> tiles [n, Tz, Ty, Tx, C...]."""
    t, kind = dev.to_device(volume)
    sp, ch = _split_shape(t.shape, ndim)
    tile = (tile,) * ndim if isinstance(tile, int) else tuple(int(x) for x in tile)
    if len(tile) != ndim or any(s % x for s, x in zip(sp, tile)):
        raise AssertionError(f'volume extents {sp} must be multiples of the tile {tile}')
    n = dev.prod(s // x for s, x in zip(sp, tile))
    out = dev.empty((n, *tile, *ch), t.dtype)
    if t.numel():
        check(lib.kmp_tiles(ndim, dev.dtype_code(t), 0, t.data_ptr(), _lib.i64x3(sp), dev.prod(ch), _lib.i64x3(tile),
                            out.data_ptr(), dev.stream()), 'tiles (split)')
    return dev.from_device(out, kind)


def tiles_to_volume(tiles, shape, ndim=3):
    """Inverse of :func:`volume_to_tiles`: tiles [n, Tz, Ty, Tx, C...] -> volume of spatial ``shape``."""
    t, kind = dev.to_device(tiles)
    tile = tuple(int(s) for s in t.shape[1:1 + ndim])
    ch = tuple(int(s) for s in t.shape[1 + ndim:])
    shape = tuple(int(s) for s in shape)
    if len(shape) != ndim or any(s % x for s, x in zip(shape, tile)):
        raise AssertionError(f'volume extents {shape} must be multiples of the tile {tile}')
    if dev.prod(s // x for s, x in zip(shape, tile)) != t.shape[0]:
        raise AssertionError(f'{t.shape[0]} tiles of {tile} do not assemble a volume of {shape}')
    out = dev.empty((*shape, *ch), t.dtype)
    if t.numel():
        check(lib.kmp_tiles(ndim, dev.dtype_code(t), 1, t.data_ptr(), _lib.i64x3(shape), dev.prod(ch),
                            _lib.i64x3(tile), out.data_ptr(), dev.stream()), 'tiles (assemble)')
    return dev.from_device(out, kind)
