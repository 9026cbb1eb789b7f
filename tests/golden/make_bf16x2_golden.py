"""Regression fixtures for the matrix-core LinearPredictor arithmetic (arith='bf16x2', kmp_bf16x2.h).

bf16x2 is not a restatement of any reference arithmetic (the reference leaves the predictor to the
caller, volume/encode_decode.py:48): it is the build's own, pinned to the oracle only within the
north star's 1e-5.  Its exact bits depend on how the products are grouped into MFMAs, so a change
of that grouping silently changes every coded map.  These fixtures record the maps and a hash of
the float32 cell values the current revision (predictors.ARITH_REV['bf16x2']) produces, so such a
change fails tests/test_gpu_linear.py::test_linear_bf16x2_golden and forces a revision bump.

Generated on the GPU (there is no bit-exact CPU model of the MFMA accumulation):
    python tests/golden/make_bf16x2_golden.py        # writes tests/golden/bf16x2_r<rev>.npz
"""

import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

# (name, ndim, padding, shape, dtype): the fused p = 1 kernel (linear3pm), the fused p = 0 kernel
# (linear3m), the generic MFMA kernel for 3D / 2D, 8- and 16-bit samples
CASES = [('v3_p1_u16_fused', 3, 1, (1, 32, 32, 32, 1), np.uint16),
         ('v3_p1_u16_generic', 3, 1, (2, 9, 10, 12, 1), np.uint16),
         ('v3_p0_u16_fused', 3, 0, (1, 16, 32, 32, 1), np.uint16),
         ('v3_p1_u8', 3, 1, (1, 8, 32, 64, 1), np.uint8),
         ('v2_p1_u16_generic', 2, 1, (2, 30, 31, 2), np.uint16)]


def case_inputs(ndim, padding, shape, dtype, seed):
    """Smooth data + noise (small residuals: the fixture compresses) and noisy-mean weights."""
    rng = np.random.default_rng(seed)
    grids = np.meshgrid(*[np.arange(s) for s in shape[1:1 + ndim]], indexing='ij')
    top = 60000 if dtype == np.uint16 else 250
    field = sum(rng.uniform(0.2, 1.0) * g / max(1, g.max()) for g in grids) / ndim
    hi = np.empty(shape, np.float64)
    for b in range(shape[0]):
        for c in range(shape[-1]):
            hi[b, ..., c] = 10 + top * field + rng.normal(0, top / 400, field.shape)
    hi = np.clip(np.round(hi), 0, np.iinfo(dtype).max).astype(dtype)
    n, k = (2 * padding + 2) ** ndim, 19 if ndim == 3 else 5
    w = (1.0 / n + rng.standard_normal((n, k)) * (0.3 / n)).astype(np.float32)
    bias = (rng.standard_normal(k) * (3.0 if dtype == np.uint8 else 50.0)).astype(np.float32)
    return hi, w, bias


def run_case(kom, ndim, padding, shape, dtype, seed):
    """(dims, maps, sha256 of the f32 cell values, the launch that coded it) for one case."""
    import oracle
    hi, w, b = case_inputs(ndim, padding, shape, dtype, seed)
    ns, ons = (kom.volume, oracle.volume) if ndim == 3 else (kom.image, oracle.image)
    enc = ns.encode_values_uint16 if dtype == np.uint16 else ns.encode_values_uint8
    pred = kom.LinearPredictor(w, b, padding, ndim, arith='bf16x2')
    lo, (maps, dims) = ns.encode(pred, enc, hi, padding=padding)
    launch = kom._lib.lib.kmp_last_launch().decode()
    window = ons.pad_neighborhood(ons.lowres_from_highres(ons.pad_highres(hi)[0]), padding)
    _, cells_f = pred.predict_cells(window, with_f32=True)
    sha = hashlib.sha256(np.ascontiguousarray(cells_f).view(np.uint32).tobytes()).hexdigest()
    return np.asarray(dims), [np.asarray(m) for m in maps], sha, launch


def main():
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    import kompressor_amd as kom
    from kompressor_amd.predictors import ARITH_REV
    rev = ARITH_REV['bf16x2']
    out = {'arith_rev': np.int32(rev)}
    for i, (name, ndim, p, shape, dtype) in enumerate(CASES):
        # generated on the generic MFMA kernel (kmp_linear.hip, unchanged since the revision's
        # introduction); the test checks the fused kernels against the same bits
        with kom._lib.option('KMP_DISABLE_LINEAR_FUSED', 1):
            dims, maps, sha, launch = run_case(kom, ndim, p, shape, dtype, 500 + i)
        out[f'{name}/dims'] = dims
        out[f'{name}/cells_sha256'] = np.array(sha)
        out[f'{name}/launch'] = np.array(launch)
        for j, m in enumerate(maps):
            out[f'{name}/map{j}'] = m
        print(name, launch, sha[:16], [m.shape for m in maps])
    path = os.path.join(HERE, f'bf16x2_r{rev}.npz')
    np.savez_compressed(path, **out)
    print('wrote', path, os.path.getsize(path), 'bytes')


if __name__ == '__main__':
    main()
