"""Regenerate the golden fixtures in this directory from the CPU oracle.

    python tests/golden/make_golden.py

Every fixture is an ``.npz`` of inputs and expected outputs (data only).  Outputs come from
``oracle`` (numpy op-for-op restatement of the reference) and, for the mean-predictor codec
cases, are cross-checked against the independent per-element restatement ``oracle.loops``
before being written.  The reference itself cannot run here (JAX absent; see oracle/__init__.py),
so these vectors pin the HIP path to the oracle, not to reference-produced outputs.
"""

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, '..', '..')))

from oracle import volume as V, image as I, predictors as P, loops as Lp, common  # noqa: E402


def ramp(shape, max_value, dtype):
    # tests/volume/test_encode_decode.py:39-41 -- arange(prod(shape)).reshape(shape) % max_value
    return (np.arange(np.prod(shape)).reshape(shape) % max_value).astype(dtype)


def rand(shape, dtype, seed):
    info = np.iinfo(dtype)
    return np.random.default_rng(seed).integers(0, int(info.max) + 1, size=shape, dtype=np.int64).astype(dtype)


CODERS = {np.dtype(np.uint8): ('uint8', V.encode_values_uint8, V.decode_values_uint8),
          np.dtype(np.uint16): ('uint16', V.encode_values_uint16, V.decode_values_uint16),
          np.dtype(np.int32): ('raw', V.encode_values_raw, V.decode_values_raw)}


def codec_case(name, hi, padding, ndim, check_loops=True):
    ns = V if ndim == 3 else I
    coder, enc, dec = CODERS[hi.dtype]
    pf = P.mean_predictions_fn(padding, ndim)
    lowres, (maps, dims) = ns.encode(pf, enc, hi, padding=padding)
    rec = ns.decode(pf, dec, lowres, (maps, dims), padding=padding)
    assert np.array_equal(rec, hi), name
    if check_loops and hi.dtype != np.int32:
        lo2, maps2, dims2 = Lp.encode_mean(hi, padding, ndim)
        assert dims2 == tuple(dims) and np.array_equal(lo2, lowres), name
        for a, b in zip(maps, maps2):
            assert np.array_equal(a, b), name
    out = {'highres': hi, 'lowres': lowres, 'dims': np.array(dims, np.int32), 'padding': np.int32(padding),
           'ndim': np.int32(ndim), 'coder': np.array(coder)}
    for i, m in enumerate(maps):
        out[f'map{i}'] = m
    np.savez_compressed(os.path.join(HERE, name + '.npz'), **out)
    print(name, hi.shape, hi.dtype, 'p=%d' % padding, 'dims', dims)


def categorical_case(name, hi, padding, ndim):
    ns = V if ndim == 3 else I
    pf = P.categorical_predictions_fn(padding, 256, ndim)
    lowres, (maps, dims) = ns.encode(pf, common.encode_categorical, hi, padding=padding)
    rec = ns.decode(pf, common.decode_categorical, lowres, (maps, dims), padding=padding)
    assert np.array_equal(rec, hi), name
    out = {'highres': hi, 'lowres': lowres, 'dims': np.array(dims, np.int32), 'padding': np.int32(padding),
           'ndim': np.int32(ndim),
           'logits': P.categorical_logits(ndim, hi.shape[ndim + 1:], 256)}
    for i, m in enumerate(maps):
        out[f'map{i}'] = m
    np.savez_compressed(os.path.join(HERE, name + '.npz'), **out)
    print(name, hi.shape, hi.dtype, 'p=%d' % padding)


def maps_from_predictions_case(name, preds, ndim):
    ns = V if ndim == 3 else I
    maps = ns.maps_from_predictions(preds)
    out = {'predictions': preds, 'ndim': np.int32(ndim)}
    for i, m in enumerate(maps):
        out[f'map{i}'] = m
    np.savez_compressed(os.path.join(HERE, name + '.npz'), **out)
    print(name, preds.shape, preds.dtype)


def main():
    # volume, the reference test shapes (tests/volume/test_encode_decode.py:39-41, :166)
    for p in (0, 1):
        codec_case(f'vol_ramp_odd_p{p}', ramp((2, 17, 17, 17, 1), 65536, np.uint16), p, 3)
        codec_case(f'vol_ramp_even_p{p}', ramp((2, 16, 16, 16, 1), 65536, np.uint16), p, 3)
    for p in (0, 1, 2):
        codec_case(f'vol_rand_mixed_p{p}', rand((2, 9, 10, 12, 1), np.uint16, 10 + p), p, 3)
    codec_case('vol_rand_u8_c3_p1', rand((2, 9, 8, 11, 3), np.uint8, 20), 1, 3)
    codec_case('vol_rand_u8_p0', rand((2, 10, 12, 32, 1), np.uint8, 21), 0, 3)
    codec_case('vol_ramp_i32_raw_p0', ramp((2, 17, 17, 17, 1), 65536, np.int32), 0, 3)
    # one metric tile (default_rng(0) uint16, 64^3), p = 0 and p = 1
    tile = rand((1, 64, 64, 64, 1), np.uint16, 0)
    codec_case('vol_tile64_p0', tile, 0, 3, check_loops=False)
    codec_case('vol_tile64_p1', tile, 1, 3, check_loops=False)
    codec_case('vol_tile_small_p0', rand((3, 16, 24, 32, 1), np.uint16, 1), 0, 3)
    codec_case('vol_tile_small_p1', rand((2, 15, 12, 16, 1), np.uint16, 2), 1, 3)
    # image, the reference test shapes (tests/image/test_encode_decode.py:39-41, :160)
    for p in (0, 1):
        codec_case(f'img_ramp_odd_p{p}', ramp((2, 17, 17, 3), 256, np.uint8), p, 2)
        codec_case(f'img_ramp_even_p{p}', ramp((2, 16, 16, 3), 256, np.uint8), p, 2)
    for p in (0, 1, 2):
        codec_case(f'img_rand_p{p}', rand((3, 33, 20, 1), np.uint8, 30 + p), p, 2)
    codec_case('img_rand_u16_c2_p1', rand((2, 30, 31, 2), np.uint16, 40), 1, 2)
    codec_case('img_tile256_p0', rand((2, 256, 256, 1), np.uint8, 0), 0, 2, check_loops=False)
    codec_case('img_ramp_i32_raw_p0', ramp((2, 17, 17, 3), 256, np.int32), 0, 2)
    # shapes eligible for the one-pass kernels (C == 1, W*itemsize % 16 == 0), odd and even H/D
    codec_case('vol_fast_u16_p2', rand((2, 11, 9, 16, 1), np.uint16, 60), 2, 3)
    codec_case('vol_fast_u8_p1', rand((3, 9, 14, 32, 1), np.uint8, 61), 1, 3)
    codec_case('img_fast_u8_p1', rand((3, 30, 32, 1), np.uint8, 62), 1, 2)
    codec_case('img_fast_u8_p0', rand((5, 33, 48, 1), np.uint8, 63), 0, 2)
    codec_case('img_fast_u16_p2', rand((2, 17, 16, 1), np.uint16, 64), 2, 2)
    # categorical rank coder (reference tests use 256 classes on uint8, :217-356)
    categorical_case('vol_categorical_p0', ramp((2, 9, 9, 9, 1), 256, np.uint8), 0, 3)
    categorical_case('img_categorical_p1', ramp((2, 17, 17, 3), 256, np.uint8), 1, 2)
    # float32 aggregation semantics of maps_from_predictions (order of adds, x0.5 / x0.25, cast)
    rng = np.random.default_rng(50)
    maps_from_predictions_case('mfp_vol_f32', rng.standard_normal((2, 3, 4, 5, 19, 2)).astype(np.float32), 3)
    maps_from_predictions_case('mfp_vol_i32', rng.integers(-2**30, 2**30, (2, 3, 2, 4, 19, 1)).astype(np.int32), 3)
    maps_from_predictions_case('mfp_vol_u16', rng.integers(0, 65536, (1, 4, 3, 2, 19, 1)).astype(np.uint16), 3)
    maps_from_predictions_case('mfp_img_f32', rng.standard_normal((2, 5, 6, 5, 3)).astype(np.float32), 2)
    maps_from_predictions_case('mfp_img_u8', rng.integers(0, 256, (2, 5, 6, 5, 1)).astype(np.uint8), 2)


if __name__ == '__main__':
    main()
