"""Codec plans replayed from HIP graphs (kompressor_amd.graphs.CodecPlan): the captured encode /
decode give exactly the eager fused results, on new inputs written into the static buffer, for
volumes (p = 0, 1, 2) and images, and replays are lossless."""

import numpy as np
import pytest
import torch

from conftest import ROOT  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('ndim,shape,dtype,p', [
    (3, (16, 64, 64, 64, 1), torch.uint16, 0),
    (3, (8, 33, 40, 64, 1), torch.uint16, 1),
    (3, (8, 64, 64, 64, 1), torch.uint16, 2),
    (2, (32, 256, 256, 1), torch.uint8, 0),
    (2, (8, 100, 128, 1), torch.uint8, 1),
    (3, (4, 32, 32, 32, 1), torch.int32, 0),
])
def test_plan_matches_eager(kom, ndim, shape, dtype, p):
    ns = kom.volume if ndim == 3 else kom.image
    name = {torch.uint16: 'uint16', torch.uint8: 'uint8', torch.int32: 'raw'}[dtype]
    enc, dec = getattr(ns, f'encode_values_{name}'), getattr(ns, f'decode_values_{name}')
    pred = kom.MeanPredictor(p, ndim)
    plan = kom.graphs.CodecPlan(pred, shape, dtype)
    gen = torch.Generator(device='cuda').manual_seed(p)
    hi = (1 << 16) if dtype == torch.uint16 else (256 if dtype == torch.uint8 else 1 << 20)
    for rep in range(3):  # new data in the static input every replay
        x = torch.randint(0, hi, shape, device='cuda', generator=gen, dtype=torch.int64).to(dtype)
        lo, (maps, dims) = plan.encode(x)
        want_lo, (want_maps, want_dims) = ns.encode(pred, enc, x, padding=p)
        assert torch.equal(lo, want_lo) and tuple(dims) == tuple(want_dims)
        assert all(torch.equal(a, b) for a, b in zip(maps, want_maps))
        assert torch.equal(plan.decode(), x)
        # the eager decode of the plan's outputs agrees too
        assert torch.equal(ns.decode(pred, dec, lo, (maps, dims), padding=p), x)
    # copy=True: fresh tensors that the next replay does not overwrite
    lo_c, (maps_c, _) = plan.encode(x, copy=True)
    rec_c = plan.decode(copy=True)
    keep = (lo_c.clone(), [m.clone() for m in maps_c], rec_c.clone())
    plan.encode(torch.zeros_like(x))
    plan.decode()
    assert lo_c.data_ptr() != plan.lowres.data_ptr() and torch.equal(lo_c, keep[0])
    assert all(torch.equal(a, b) for a, b in zip(maps_c, keep[1])) and torch.equal(rec_c, keep[2])


def _torch_predictions_fn(kom, ndim, padding):
    """A capture-safe network-like predictions_fn: float32 features -> scaled mean + per-channel
    offsets -> maps_from_predictions; device ops only, no host synchronisation."""
    ns = kom.volume if ndim == 3 else kom.image
    k = 19 if ndim == 3 else 5

    def fn(lowres):
        features = ns.features_from_lowres(lowres, padding).to(torch.float32)
        pred = torch.mean(features, dim=ndim + 1, keepdim=True) * 1.37 - 40.25
        pred = pred.repeat_interleave(k, dim=ndim + 1)
        pred = pred + torch.linspace(-3.7, 2.9, k, device=pred.device).reshape(
            *([1] * (ndim + 1)), k, *([1] * (pred.dim() - ndim - 2)))
        return ns.maps_from_predictions(pred.contiguous())

    return fn


@pytest.mark.parametrize('ndim,shape,dtype,p,kind', [
    (3, (16, 64, 64, 64, 1), torch.uint16, 0, 'wrapped'),
    (3, (8, 33, 40, 64, 1), torch.uint16, 1, 'torch'),
    (3, (4, 32, 32, 32, 2), torch.uint8, 2, 'wrapped'),
    (2, (16, 256, 256, 1), torch.uint8, 1, 'torch'),
    (2, (8, 100, 128, 1), torch.uint16, 0, 'wrapped'),
])
def test_callback_plan_matches_eager(kom, ndim, shape, dtype, p, kind):
    """CodecPlan of an opaque predictions_fn (the callback path captured into graphs): a built-in
    predictor behind a lambda, or a float32 torch-op predictor; every replay on new data gives the
    eager callback path's lowres / maps bit for bit and decodes losslessly."""
    ns = kom.volume if ndim == 3 else kom.image
    name = {torch.uint16: 'uint16', torch.uint8: 'uint8'}[dtype]
    enc, dec = getattr(ns, f'encode_values_{name}'), getattr(ns, f'decode_values_{name}')
    if kind == 'wrapped':
        pred = kom.MeanPredictor(p, ndim)
        fn = lambda lowres: pred(lowres)  # noqa: E731
    else:
        fn = _torch_predictions_fn(kom, ndim, p)
    plan = kom.graphs.CodecPlan(fn, shape, dtype, padding=p)
    assert not plan.fused
    gen = torch.Generator(device='cuda').manual_seed(7 + p)
    hi = (1 << 16) if dtype == torch.uint16 else 256
    for rep in range(3):
        x = torch.randint(0, hi, shape, device='cuda', generator=gen, dtype=torch.int64).to(dtype)
        lo, (maps, dims) = plan.encode(x)
        want_lo, (want_maps, want_dims) = ns.encode(fn, enc, x, padding=p)
        assert torch.equal(lo, want_lo) and tuple(dims) == tuple(want_dims)
        assert all(torch.equal(a, b) for a, b in zip(maps, want_maps))
        assert torch.equal(plan.decode(), x)
        assert torch.equal(ns.decode(fn, dec, lo, (maps, dims), padding=p), x)


def test_plan_argument_checks(kom):
    with pytest.raises(ValueError):
        kom.graphs.CodecPlan(lambda lowres: lowres, (2, 16, 16, 16, 1), torch.uint16)  # no padding
    with pytest.raises(ValueError):
        kom.graphs.CodecPlan(kom.MeanPredictor(1, 3), (2, 16, 16, 16, 1), torch.uint16, padding=0)
