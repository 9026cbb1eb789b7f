"""Oracle (test infrastructure only): an independent per-element restatement, pure Python loops.

Written from the reference's arithmetic, not from its op sequence, to cross-check the numpy
op-for-op restatement (``oracle.volume`` / ``oracle.image``) on small inputs.  It treats an
N-d (N = 2 or 3) highres array as 2^N parity classes of a "block" grid:

* the even-dim reflect pad (volume/utils.py:226-237) only ever supplies the far lowres node,
  ``highres[n] -> highres[n - 2]``;
* a cell ``c`` (per axis ``0 .. L-2``, L = padded lowres length) predicts from the lowres nodes
  ``c-p .. c+p+1`` (symmetric mirror outside ``[0, L)``; volume/utils.py:199-218);
* the mean predictor (tests/volume/test_encode_decode.py:46-53) is ``floor(sum / (2p+2)^N)``;
* a map of parity ``(p_a)`` at output ``o`` aggregates the cells ``{o}`` on odd axes and
  ``{o-1, o} ∩ [0, L-1)`` on even axes and divides by their count -- the ×0.5 / ×0.25
  normalisation of volume/utils.py:83-155 -- truncating;
* output extents are ``L-1`` on odd axes and ``L - dims`` on even axes (trim_maps, :270-276);
* the residual is ``(gt - pred) mod 2^bits`` (utils.py:38-55).
Slow: use only for inputs of a few thousand elements.
"""

from itertools import product

import numpy as np

from .common import sym_index


def _geometry(shape, ndim):
    n = shape[1:ndim + 1]
    dims = tuple((s + 1) % 2 for s in n)
    L = tuple((s + d + 1) // 2 for s, d in zip(n, dims))
    return n, dims, L


def _parities(ndim):
    # Map order of the reference: 3D LR, UD, FB, C, Z, Y, X (volume/utils.py:161-169);
    # 2D LR, UD, C (image/utils.py:92-94).
    if ndim == 3:
        return [(1, 1, 0), (1, 0, 1), (0, 1, 1), (1, 1, 1), (1, 0, 0), (0, 1, 0), (0, 0, 1)]
    return [(1, 0), (0, 1), (1, 1)]


class _Grid:
    def __init__(self, lowres_get, L, padding, ndim):
        self.lowres_get, self.L, self.p, self.ndim = lowres_get, L, padding, ndim
        self.cache = {}

    def mean(self, b, cell, c):
        key = (b, cell, c)
        if key not in self.cache:
            k = 2 * self.p + 2
            total = 0
            for off in product(range(k), repeat=self.ndim):
                idx = tuple(sym_index(ci - self.p + o, Li) for ci, o, Li in zip(cell, off, self.L))
                total += int(self.lowres_get(b, idx, c))
            self.cache[key] = total // (k ** self.ndim)
        return self.cache[key]

    def prediction(self, b, parity, out, c):
        choices = []
        for par, o, Li in zip(parity, out, self.L):
            ncell = Li - 1
            choices.append([o] if par else [q for q in (o - 1, o) if 0 <= q < ncell])
        cells = list(product(*choices))
        return sum(self.mean(b, cell, c) for cell in cells) // len(cells)


def encode_mean(highres, padding, ndim):
    """Mean-predictor encode with the modular coder of the input's bit width.
    Returns ``(lowres, maps, dims)`` like the reference's ``encode``."""
    h = np.asarray(highres)
    bits = h.dtype.itemsize * 8
    mod = 1 << bits
    n, dims, L = _geometry(h.shape, ndim)
    B = h.shape[0]
    chan = h.shape[ndim + 1:]
    hflat = h.reshape(B, *n, -1)
    C = hflat.shape[-1]

    def hv(b, idx, c):
        src = tuple(i if i < s else 2 * (s - 1) - i for i, s in zip(idx, n))
        return int(hflat[(b, *src, c)])

    def lowres_get(b, idx, c):
        return hv(b, tuple(2 * i for i in idx), c)

    grid = _Grid(lowres_get, L, padding, ndim)
    lo_ext = tuple(Li - d for Li, d in zip(L, dims))
    lowres = np.zeros((B, *lo_ext, C), h.dtype)
    for b, c in product(range(B), range(C)):
        for idx in product(*[range(e) for e in lo_ext]):
            lowres[(b, *idx, c)] = lowres_get(b, idx, c)
    maps = []
    for parity in _parities(ndim):
        ext = tuple((Li - 1) if par else (Li - d) for par, Li, d in zip(parity, L, dims))
        m = np.zeros((B, *ext, C), h.dtype)
        for b, c in product(range(B), range(C)):
            for o in product(*[range(e) for e in ext]):
                gt = hv(b, tuple(2 * oi + par for oi, par in zip(o, parity)), c)
                m[(b, *o, c)] = (gt - grid.prediction(b, parity, o, c)) % mod
        maps.append(m.reshape(B, *ext, *chan))
    return lowres.reshape(B, *lo_ext, *chan), tuple(maps), dims


def decode_mean(lowres, maps, dims, padding, ndim):
    """Mean-predictor decode: rebuild the highres from the trimmed lowres and residual maps."""
    lo = np.asarray(lowres)
    bits = lo.dtype.itemsize * 8
    mod = 1 << bits
    B = lo.shape[0]
    chan = lo.shape[ndim + 1:]
    lo_ext = lo.shape[1:ndim + 1]
    L = tuple(e + d for e, d in zip(lo_ext, dims))
    n = tuple(2 * Li - 1 - d for Li, d in zip(L, dims))
    loflat = lo.reshape(B, *lo_ext, -1)
    C = loflat.shape[-1]

    def lowres_get(b, idx, c):
        # decode's pad_lowres is a symmetric pad by dims (volume/utils.py:240-244)
        src = tuple(sym_index(i, e) for i, e in zip(idx, lo_ext))
        return int(loflat[(b, *src, c)])

    grid = _Grid(lowres_get, L, padding, ndim)
    out = np.zeros((B, *n, C), lo.dtype)
    for b, c in product(range(B), range(C)):
        for idx in product(*[range(e) for e in lo_ext]):
            out[(b, *(2 * i for i in idx), c)] = loflat[(b, *idx, c)]
    for parity, m in zip(_parities(ndim), maps):
        mf = np.asarray(m).reshape(B, *np.asarray(m).shape[1:ndim + 1], -1)
        ext = mf.shape[1:ndim + 1]
        for b, c in product(range(B), range(C)):
            for o in product(*[range(e) for e in ext]):
                pos = tuple(2 * oi + par for oi, par in zip(o, parity))
                if all(pi < ni for pi, ni in zip(pos, n)):
                    out[(b, *pos, c)] = (grid.prediction(b, parity, o, c) + int(mf[(b, *o, c)])) % mod
    return out.reshape(B, *n, *chan)
