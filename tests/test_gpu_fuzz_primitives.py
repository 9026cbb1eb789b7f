"""Randomised parity sweep of the geometry primitives the reference exports
(volume/utils.py:29-276, image/utils.py:26-133): seeded random shapes (odd and even extents, 1-3
channels), every sample dtype, padding 0-3, each primitive's HIP kernel against the oracle's
restatement, bit for bit.  maps_from_predictions runs on float32, int32 and the sample dtype (its
f32 aggregation in the reference's add order).  200 cases by default (KMP_FUZZ_CASES)."""

import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DTYPES = [np.uint8, np.uint16, np.int32, np.uint32, np.float32]


def _rand(rng, shape, dtype):
    if dtype == np.float32:
        return (rng.standard_normal(shape) * 1000).astype(np.float32)
    info = np.iinfo(dtype)
    return rng.integers(int(info.min), int(info.max) + 1, size=shape, dtype=np.int64).astype(dtype)


def _eq(a, b, what):
    a = np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape and a.dtype == b.dtype, (what, a.shape, b.shape, a.dtype, b.dtype)
    assert a.tobytes() == b.tobytes(), what  # bitwise, so float NaN / -0 count


_SEED0 = int(os.environ.get('KMP_FUZZ_SEED0', '0'))  # first case (later sweeps draw new cases)


@pytest.mark.parametrize('seed', range(_SEED0, _SEED0 + int(os.environ.get('KMP_FUZZ_CASES', '200'))))
def test_random_primitives_match_oracle(kom, seed):
    import oracle
    rng = np.random.default_rng(5000 + seed)
    ndim = 3 if seed % 2 == 0 else 2
    ns, ons = (kom.volume.utils, oracle.volume) if ndim == 3 else (kom.image.utils, oracle.image)
    dtype = DTYPES[int(rng.integers(0, len(DTYPES)))]
    p = int(rng.integers(0, 4))
    C = int(rng.choice([1, 1, 1, 2, 3]))
    sp = [int(rng.integers(2, 24 if ndim == 3 else 70)) for _ in range(ndim)]
    x = _rand(rng, (int(rng.integers(1, 4)), *sp, C), dtype)
    info = f'ndim={ndim} dtype={np.dtype(dtype).name} p={p} shape={x.shape}'

    hp, dims = ns.pad_highres(x)
    ohp, odims = ons.pad_highres(x)
    _eq(hp, ohp, ('pad_highres', info))
    assert tuple(dims) == tuple(odims), info
    if min(ohp.shape[1:1 + ndim]) < 3:
        return  # the reference's encode would reject it; the remaining primitives need 3+ nodes
    lo, olo = ns.lowres_from_highres(ohp), ons.lowres_from_highres(ohp)
    _eq(lo, olo, ('lowres_from_highres', info))
    maps, omaps = ns.maps_from_highres(ohp), ons.maps_from_highres(ohp)
    for i, (m, om) in enumerate(zip(maps, omaps)):
        _eq(m, om, ('maps_from_highres', i, info))
    _eq(ns.targets_from_highres(ohp), ons.targets_from_highres(ohp), ('targets_from_highres', info))
    win = ons.pad_neighborhood(olo, p)  # features_from_lowres takes the padded window (utils.py:199-210)
    _eq(ns.pad_neighborhood(olo, p), win, ('pad_neighborhood', info))
    _eq(ns.features_from_lowres(win, p), ons.features_from_lowres(win, p), ('features_from_lowres', info))
    _eq(ns.highres_from_lowres_and_maps(olo, omaps), ons.highres_from_lowres_and_maps(olo, omaps),
        ('highres_from_lowres_and_maps', info))
    # trims and their inverse pads with this input's dims
    tlo, otlo = ns.trim(olo, odims), ons.trim(olo, odims)
    _eq(tlo, otlo, ('trim', info))
    tmaps, otmaps = ns.trim_maps(omaps, odims), ons.trim_maps(omaps, odims)
    for i, (m, om) in enumerate(zip(tmaps, otmaps)):
        _eq(m, om, ('trim_maps', i, info))
    _eq(ns.pad_lowres(otlo, odims), ons.pad_lowres(otlo, odims), ('pad_lowres', info))
    for i, (m, om) in enumerate(zip(ns.pad_maps(otmaps, odims), ons.pad_maps(otmaps, odims))):
        _eq(m, om, ('pad_maps', i, info))
    # maps_from_predictions on per-cell predictions [B, cells..., K, C]
    K = 19 if ndim == 3 else 5
    cells = [s - 1 for s in olo.shape[1:1 + ndim]]
    pdt = [np.float32, np.int32, dtype][int(rng.integers(0, 3))]
    preds = _rand(rng, (olo.shape[0], *cells, K, C), pdt)
    for i, (m, om) in enumerate(zip(ns.maps_from_predictions(preds), ons.maps_from_predictions(preds))):
        _eq(m, om, ('maps_from_predictions', np.dtype(pdt).name, i, info))
