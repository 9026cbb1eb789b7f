#!/usr/bin/env python3
"""Throughput of every SURVEY.md §8(a) row on the GPU, against the HBM roofline, with the CPU
oracle timed beside it on a small sample of the same workload.

    python tools/bench_rows.py [--reps N] [--rows name,name,...] [--no-cpu]

One JSON line per row: {"row", "what", "GBps", "frac", "us", "algo_bytes", "cpu_GBps", "cpu_sample"}.
``GBps`` = algorithmic bytes per call (inputs read + outputs written once) over the
HIP-event time of ``reps`` back-to-back calls on device-resident inputs.  bench.py remains the
headline (C3); this covers the secondary rows (p = 1, 2, LinearPredictor, chunked drivers, the
reference-style callback path, categorical coder, primitives, tiling).
"""

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

PEAK = 8000.0


def gpu_time(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / 1e3


def cpu_time(fn, budget=3.0):
    t = time.perf_counter()
    fn()
    first = time.perf_counter() - t
    n = max(1, min(5, int(budget / max(first, 1e-3))))
    t = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t) / n


def rand(shape, dtype, seed=0):
    info = np.iinfo(dtype)
    return np.random.default_rng(seed).integers(0, int(info.max) + 1, size=shape, dtype=np.int64).astype(dtype)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--rows', default='')
    ap.add_argument('--no-cpu', action='store_true')
    args = ap.parse_args()
    want = set(filter(None, args.rows.split(',')))

    import kompressor_amd as kom
    from kompressor_amd import _nd
    import oracle
    from oracle import predictors as OP
    torch.cuda.set_device(0)

    vol_h = rand((512, 64, 64, 64, 1), np.uint16)
    vol = torch.from_numpy(vol_h).cuda()
    img_h = rand((1024, 256, 256, 1), np.uint8)
    img = torch.from_numpy(img_h).cuda()
    V, I = kom.volume, kom.image
    OV, OI = oracle.volume, oracle.image
    raw_v, raw_i = vol.numel() * 2, img.numel()

    def emit(row, what, algo, t, cpu=None):
        line = {'row': row, 'what': what, 'GBps': round(algo / t / 1e9, 1), 'frac': round(algo / t / 1e9 / PEAK, 4),
                'us': round(t * 1e6, 2), 'algo_bytes': int(algo)}
        if cpu:
            line['cpu_GBps'] = round(cpu[0], 5)
            line['cpu_sample'] = cpu[1]
        print(json.dumps(line), flush=True)

    def cpu_codec(ons, pf, enc, dec, sample, padding):
        if args.no_cpu:
            return None

        def rnd():
            lo, e = ons.encode(pf, enc, sample, padding=padding)
            ons.decode(pf, dec, lo, e, padding=padding)
        t = cpu_time(rnd)
        return sample.nbytes * 2 * 2 / t / 1e9, f'{sample.shape[0]} tiles, oracle encode+decode, 1 thread'

    def codec_rows(tag, ns, ons, x, xh, pred, opf, enc, dec, oenc, odec, padding, raw, ndim, with_cpu=True):
        if want and tag not in want:
            return
        coder = _nd.NATURAL_CODER[x.dtype]
        lo, maps, dims = _nd._alloc_encoded(x, coder, ndim)
        rec = torch.empty_like(x)
        ws = torch.empty(max(1, _nd.workspace_bytes(x, pred, ndim)), dtype=torch.uint8, device='cuda')
        fe = lambda: _nd.fused_encode_into(x, pred, coder, lo, maps, ndim, workspace=ws)  # noqa: E731
        fd = lambda: _nd.fused_decode_into(lo, maps, dims, pred, coder, rec, ndim, workspace=ws)  # noqa: E731
        fe(), fd()
        torch.cuda.synchronize()
        assert torch.equal(rec, x), tag
        te, td = gpu_time(fe, args.reps), gpu_time(fd, args.reps)
        cpu = cpu_codec(ons, opf, oenc, odec, xh[:2], padding) if with_cpu else None
        emit(tag + ':encode', f'fused encode {pred!r}', 2 * raw, te, cpu)
        emit(tag + ':decode', f'fused decode {pred!r}', 2 * raw, td)

    for p in (0, 1, 2):
        codec_rows(f'volume_mean_p{p}', V, OV, vol, vol_h, kom.MeanPredictor(p, 3), OP.mean_predictions_fn(p, 3),
                   V.encode_values_uint16, V.decode_values_uint16, OV.encode_values_uint16, OV.decode_values_uint16,
                   p, raw_v, 3)
    for p in (0, 1, 2):
        codec_rows(f'image_mean_p{p}', I, OI, img, img_h, kom.MeanPredictor(p, 2), OP.mean_predictions_fn(p, 2),
                   I.encode_values_uint8, I.decode_values_uint8, OI.encode_values_uint8, OI.decode_values_uint8,
                   p, raw_i, 2)
    rng = np.random.default_rng(1)
    for p in (0, 1):
        n = (2 * p + 2) ** 3
        w = (1.0 / n + rng.standard_normal((n, 19)) * (0.3 / n)).astype(np.float32)
        b = np.zeros(19, np.float32)
        codec_rows(f'volume_linear_p{p}', V, OV, vol, vol_h, kom.LinearPredictor(w, b, p, 3, arith='f32'),
                   OP.linear_predictions_fn(p, w, b, 3), V.encode_values_uint16, V.decode_values_uint16,
                   OV.encode_values_uint16, OV.decode_values_uint16, p, raw_v, 3)

    rng_bf = np.random.default_rng(1)
    for p in (0, 1):  # the matrix-core arithmetic (arith='bf16x2'), the same weights as the f32 rows
        n = (2 * p + 2) ** 3
        w = (1.0 / n + rng_bf.standard_normal((n, 19)) * (0.3 / n)).astype(np.float32)
        b = np.zeros(19, np.float32)
        codec_rows(f'volume_linear_bf16x2_p{p}', V, OV, vol, vol_h, kom.LinearPredictor(w, b, p, 3, arith='bf16x2'),
                   None, V.encode_values_uint16, V.decode_values_uint16, None, None, p, raw_v, 3, with_cpu=False)

    # uint8 volumes at C3 geometry (512 tiles of 64^3), p = 1: the f32 chain vs the matrix cores
    # (linear3pm's u8 form, the 'auto' default since round 6)
    if not want or want & {'volume_linear_u8_p1', 'volume_linear_bf16x2_u8_p1'}:
        vol8_h = rand((512, 64, 64, 64, 1), np.uint8)
        vol8 = torch.from_numpy(vol8_h).cuda()
        w = (1.0 / 64 + np.random.default_rng(2).standard_normal((64, 19)) * (0.3 / 64)).astype(np.float32)
        b = np.zeros(19, np.float32)
        for tag, ar in (('volume_linear_u8_p1', 'f32'), ('volume_linear_bf16x2_u8_p1', 'bf16x2')):
            codec_rows(tag, V, OV, vol8, vol8_h, kom.LinearPredictor(w, b, 1, 3, arith=ar), None,
                       V.encode_values_uint8, V.decode_values_uint8, None, None, 1, vol8.numel(), 3, with_cpu=False)
        del vol8

    for p in (0,):
        n = (2 * p + 2) ** 2
        w = (1.0 / n + rng.standard_normal((n, 5)) * (0.3 / n)).astype(np.float32)
        b = np.zeros(5, np.float32)
        codec_rows(f'image_linear_p{p}', I, OI, img, img_h, kom.LinearPredictor(w, b, p, 2, arith='f32'),
                   OP.linear_predictions_fn(p, w, b, 2), I.encode_values_uint8, I.decode_values_uint8,
                   OI.encode_values_uint8, OI.decode_values_uint8, p, raw_i, 2)

    # ONE 512^3 volume as a single array (global-volume mode on one GPU: 256 outputs per row)
    if not want or 'volume_global' in want:
        g = vol.view(8, 8, 8, 64, 64, 64).permute(0, 3, 1, 4, 2, 5).reshape(1, 512, 512, 512, 1)
        codec_rows('volume_global', V, OV, g, None, kom.MeanPredictor(0, 3), None, V.encode_values_uint16,
                   V.decode_values_uint16, None, None, 0, raw_v, 3, with_cpu=False)
        del g

    # chunked drivers (encode_decode_chunk.py:33-117) at C3, chunk 32 (the reference default)
    if not want or 'volume_chunks' in want:
        pred = kom.MeanPredictor(0, 3)
        lo, (maps, dims) = V.encode(pred, V.encode_values_uint16, vol)
        te = gpu_time(lambda: V.encode_chunks(pred, V.encode_values_uint16, vol, chunk=32), args.reps)
        td = gpu_time(lambda: V.decode_chunks(pred, V.decode_values_uint16, lo, (maps, dims), chunk=32), args.reps)
        emit('volume_chunks:encode', 'encode_chunks chunk=32, fused region launches', 2 * raw_v, te)
        emit('volume_chunks:decode', 'decode_chunks chunk=32, fused region launches', 2 * raw_v, td)

    # the callback path: an opaque predictions_fn (here the mean predictor's primitive) with the
    # built-in coder -- window gather, predictions_fn, one fused coder launch (kmp_callback.hip)
    if not want or 'volume_callback' in want:
        pred = kom.MeanPredictor(0, 3)
        cb = lambda lowres: pred(lowres)  # noqa: E731  (not recognised as fused: the reference's step sequence)
        for nt in (512, 128):  # the whole C3 batch (GPU-bound), and 128 tiles (host-bound, ~0.1 ms per call)
            sub = vol[:nt]
            lo, (maps, dims) = V.encode(cb, V.encode_values_uint16, sub)
            te = gpu_time(lambda: V.encode(cb, V.encode_values_uint16, sub), args.reps)
            td = gpu_time(lambda: V.decode(cb, V.decode_values_uint16, lo, (maps, dims)), args.reps)
            tag = 'volume_callback' if nt == 512 else f'volume_callback_{nt}'
            emit(tag + ':encode', f'callback encode, {nt} tiles (window, opaque predictions_fn, fused coder)',
                 sub.numel() * 4, te)
            emit(tag + ':decode', f'callback decode, {nt} tiles (window, opaque predictions_fn, fused coder)',
                 sub.numel() * 4, td)
            del lo, maps

    # the callback path with float32 prediction maps (a network's output; the coder reads int32(pred)):
    # the stand-in writes float32 maps itself (MeanPredictor(maps_dtype=float32), one launch, as a
    # network's last layer would) and the fused coder reads them directly
    # (kmp_*_with_predictions_typed); '_cast' is the round-2 stand-in (sample-dtype maps + 7 torch
    # .float() conversions, 47 us each); '_steps' the same call with an opaque coder, i.e. the
    # reference's step sequence
    if not want or 'volume_callback_f32' in want:
        pred32 = kom.MeanPredictor(0, 3, maps_dtype=torch.float32)
        pred = kom.MeanPredictor(0, 3)
        cbf = lambda lowres: pred32(lowres)  # noqa: E731
        cbc = lambda lowres: [m.float() for m in pred(lowres)]  # noqa: E731
        encs, decs = V.encode_values_uint16, V.decode_values_uint16
        for tag, fn, enc, dec in (('volume_callback_f32', cbf, encs, decs),
                                  ('volume_callback_f32_cast', cbc, encs, decs),
                                  ('volume_callback_f32_steps', cbf, lambda a, b: encs(a, b), lambda a, b: decs(a, b))):
            lo, (maps, dims) = V.encode(fn, enc, vol)
            assert torch.equal(V.decode(fn, dec, lo, (maps, dims)), vol), tag
            te = gpu_time(lambda: V.encode(fn, enc, vol), args.reps)
            td = gpu_time(lambda: V.decode(fn, dec, lo, (maps, dims)), args.reps)
            what = {'volume_callback_f32': 'predictor writes float32, fused coder',
                    'volume_callback_f32_cast': 'sample-dtype maps + torch .float(), fused coder',
                    'volume_callback_f32_steps': "the reference's step sequence"}[tag]
            emit(tag + ':encode', f'callback encode, 512 tiles, float32 prediction maps, {what}', vol.numel() * 4, te)
            emit(tag + ':decode', f'callback decode, 512 tiles, float32 prediction maps, {what}', vol.numel() * 4, td)
            del lo, maps

    # categorical rank coder (utils.py:58-111): 1M elements x 256 float32 logits
    if not want or 'categorical' in want:
        n, L = 1 << 20, 256
        logits = torch.rand((n, L), device='cuda')
        gt = torch.from_numpy(rand((n,), np.uint8)).cuda()
        enc = kom.volume.encode_categorical(logits, gt)
        te = gpu_time(lambda: kom.volume.encode_categorical(logits, gt), args.reps)
        td = gpu_time(lambda: kom.volume.decode_categorical(logits, enc), args.reps)
        cpu = None
        if not args.no_cpu:
            lh, gh = logits[:4096].cpu().numpy(), gt[:4096].cpu().numpy()
            t = cpu_time(lambda: oracle.common.encode_categorical(lh, gh))
            cpu = (4096 * (L * 4 + 2) / t / 1e9, '4096 elements, oracle stable argsort, 1 thread')
        emit('categorical:encode', 'rank coder encode, L=256', n * (L * 4 + 2), te, cpu)
        emit('categorical:decode', 'rank coder decode, L=256, uniform random ranks', n * (L * 4 + 2), td)
        small = torch.randint(0, 4, (n,), device='cuda', dtype=torch.uint8)  # a good predictor's ranks
        ts = gpu_time(lambda: kom.volume.decode_categorical(logits, small), args.reps)
        emit('categorical:decode_small_ranks', 'rank coder decode, L=256, ranks < 4', n * (L * 4 + 2), ts)

    # bit-plane container on the coded maps of a smooth C3-shaped volume
    if not want or 'packing' in want:
        zz, yy, xx = torch.meshgrid(*[torch.arange(512, device='cuda', dtype=torch.float32)] * 3, indexing='ij')
        sm = (20000 + 8000 * torch.sin(xx / 23.0) * torch.cos(yy / 17.0) + 6000 * torch.sin(zz / 29.0))
        sm = (sm + torch.randint(-2, 3, sm.shape, device='cuda')).to(torch.int32).to(torch.uint16)
        del zz, yy, xx
        tiles = sm.view(8, 64, 8, 64, 8, 64).permute(0, 2, 4, 1, 3, 5).reshape(512, 64, 64, 64, 1).contiguous()
        del sm
        pred = kom.MeanPredictor(0, 3)
        lo, (maps, dims) = V.encode(pred, V.encode_values_uint16, tiles)
        m = maps[3]  # the C map: 32 MiB of u16 residuals
        blob = kom.packing.pack(m)
        assert torch.equal(kom.packing.unpack(blob), m)
        coded = sum(kom.packing.pack(a).numel() for a in (lo, *maps))
        tp = gpu_time(lambda: kom.packing.pack(m), args.reps)
        tu = gpu_time(lambda: kom.packing.unpack(blob), args.reps)
        ratio = round(tiles.numel() * 2 / coded, 3)
        emit('packing:pack', f'bit-plane pack of a 32 MiB coded map (whole volume ratio {ratio}x)',
             m.numel() * 2 + blob.numel(), tp)
        emit('packing:unpack', 'bit-plane unpack of the same map', m.numel() * 2 + blob.numel(), tu)
        # the device chains alone (C-ABI on preallocated buffers, no header and no host sync):
        # widths + scan + pack, and scan + unpack
        from kompressor_amd import _device as kdev
        from kompressor_amd._lib import lib as klib
        n, code = m.numel(), kdev.dtype_code(m)
        nb = int(klib.kmp_pack_blocks(n))
        ws = torch.empty(int(klib.kmp_pack_workspace_bytes(n)), dtype=torch.uint8, device='cuda')
        wd = torch.empty(max(nb, 1), dtype=torch.uint8, device='cuda')
        pay = torch.empty(nb * 64 * 2, dtype=torch.uint8, device='cuda')
        out = torch.empty_like(m)

        def pack_dev():
            klib.kmp_pack_plan(code, m.data_ptr(), n, wd.data_ptr(), ws.data_ptr(), kdev.stream())
            klib.kmp_pack(code, m.data_ptr(), n, wd.data_ptr(), ws.data_ptr(), pay.data_ptr(), kdev.stream())

        def unpack_dev():
            klib.kmp_unpack_plan(wd.data_ptr(), n, ws.data_ptr(), kdev.stream())
            klib.kmp_unpack(code, pay.data_ptr(), n, wd.data_ptr(), ws.data_ptr(), out.data_ptr(), kdev.stream())

        pack_dev()
        unpack_dev()
        torch.cuda.synchronize()
        assert torch.equal(out, m)
        emit('packing:pack_device', 'widths + scan + pack kernels of the same map (no header, no host sync)',
             m.numel() * 2 + blob.numel(), gpu_time(pack_dev, args.reps))
        emit('packing:unpack_device', 'scan + unpack kernels of the same map', m.numel() * 2 + blob.numel(),
             gpu_time(unpack_dev, args.reps))
        del tiles, lo, maps

    # Rice entropy coder (kmp_rice.hip, bundle v2) vs the bit-plane format on structured C3-shaped
    # volumes: a smooth 512^3 field + Gaussian noise of std 1 / 4 / 16, tiled 64^3, MeanPredictor(0)
    # maps.  Ratio bar (tests/test_ratio.py): the order-0 entropy of the residual maps, and zlib-6 /
    # lzma-6 against Rice on the same bytes of a 16-tile sample; the container's file ratio with one
    # pyramid level and with levels='auto'
    if not want or 'rice' in want:
        import lzma
        import tempfile
        import zlib
        from kompressor_amd import packing as kpk
        zz, yy, xx = torch.meshgrid(*[torch.arange(512, device='cuda', dtype=torch.float32)] * 3, indexing='ij')
        field = (torch.sin(xx / 41.0) * torch.cos(yy / 29.0) + torch.sin(zz / 53.0 + xx / 97.0)
                 + 1.5 * torch.exp(-((xx - 200) ** 2 + (yy - 300) ** 2 + (zz - 250) ** 2) / (2 * 90.0 ** 2)))
        field = 4000 + 9000 * (field - field.min()) / (field.max() - field.min())
        del zz, yy, xx
        pred = kom.MeanPredictor(0, 3)
        gen = torch.Generator(device='cuda').manual_seed(0)
        for noise in (1.0, 4.0, 16.0):
            nvol = (field + noise * torch.randn(field.shape, device='cuda', generator=gen)).round().clamp(0, 65535)
            vol512 = nvol.to(torch.int32).to(torch.uint16)
            del nvol
            tiles = vol512.view(8, 64, 8, 64, 8, 64).permute(0, 2, 4, 1, 3, 5).reshape(512, 64, 64, 64, 1).contiguous()
            lo, (maps, dims) = V.encode(pred, V.encode_values_uint16, tiles)
            raw = tiles.numel() * 2
            b_r = kom.packing.pack_encoded(lo, (maps, dims), 'rice')
            b_p = kom.packing.pack_encoded(lo, (maps, dims), 'planes')
            lo2, (maps2, _) = kom.packing.unpack_encoded(b_r)
            assert torch.equal(lo2, lo) and all(torch.equal(a, b) for a, b in zip(maps2, maps))
            t_enc = gpu_time(lambda: kom.packing.pack_encoded(lo, (maps, dims), 'rice'), args.reps)
            t_dec = gpu_time(lambda: kom.packing.unpack_encoded(b_r), args.reps)
            hb = b_r[:4096].cpu().numpy().tobytes()
            t_enc_dev = gpu_time(lambda: kpk._rice_encode_launch((lo, *maps), dims), args.reps)
            t_dec_dev = gpu_time(lambda: kpk._rice_decode_launch(b_r, hb), args.reps)
            # order-0 entropy of the maps' residual samples (all 7 maps)
            res = torch.cat([m.reshape(-1) for m in maps]).view(torch.int16).to(torch.int32) & 0xffff
            cnt = torch.bincount(res, minlength=65536).double()
            pr = cnt[cnt > 0] / res.numel()
            h0 = float(-(pr * torch.log2(pr)).sum())
            # zlib / lzma vs Rice on the same bytes: the maps of the first 16 tiles (3.7 MB)
            sample = [m[:16].contiguous() for m in maps]
            sb = torch.cat([m.reshape(-1) for m in sample]).cpu().numpy().tobytes()
            ns = sum(m.numel() for m in sample)
            rice_s = kom.packing.pack_encoded(sample[0], (tuple(sample[1:]), dims), 'rice').numel()
            # container files: one level vs levels='auto' (the whole volume as 512 tiles)
            with tempfile.TemporaryDirectory() as td:
                f1 = kom.container.compress(td + '/l1.kmp', tiles, pred, levels=1)
                fa = kom.container.compress(td + '/la.kmp', tiles, pred, levels='auto')
            mapb = sum(m.numel() for m in maps) * 2
            line = {'row': f'rice:noise{int(noise)}', 'what': f'structured 512^3 u16 (smooth field + N(0, {noise}^2)), '
                                                             f'512 x 64^3, MeanPredictor(0)',
                    'ratio_rice': round(raw / b_r.numel(), 3), 'ratio_planes': round(raw / b_p.numel(), 3),
                    'bits_per_voxel_rice': round(8 * b_r.numel() / tiles.numel(), 3),
                    'bits_per_voxel_planes': round(8 * b_p.numel() / tiles.numel(), 3),
                    'residual_bits': {'H0': round(h0, 3), 'rice_all_maps': None,
                                      'sample_16_tiles': {'rice': round(8 * rice_s / ns, 3),
                                                          'zlib6': round(8 * len(zlib.compress(sb, 6)) / ns, 3),
                                                          'lzma6': round(8 * len(lzma.compress(sb, preset=6)) / ns, 3)}},
                    'file_ratio': {'levels_1': round(f1['ratio'], 3), 'levels_auto': round(fa['ratio'], 3),
                                   'auto_levels': fa['levels']},
                    'pack_encoded_ms': round(t_enc * 1e3, 3), 'unpack_encoded_ms': round(t_dec * 1e3, 3),
                    'pack_device_us': round(t_enc_dev * 1e6, 1), 'unpack_device_us': round(t_dec_dev * 1e6, 1),
                    'pack_encoded_GBps_raw': round(raw / t_enc / 1e9, 1),
                    'unpack_encoded_GBps_raw': round(raw / t_dec / 1e9, 1)}
            # the residual maps' share of the bundle (lowres excluded): bits per residual sample
            lo_only = kom.packing.pack(lo, 'rice').numel()
            line['residual_bits']['rice_all_maps'] = round(8 * (b_r.numel() - lo_only) / (mapb // 2), 3)
            print(json.dumps(line), flush=True)
            # device chains against HBM: the encode reads the 8 arrays once and writes the bundle,
            # the decode reads the bundle and writes the 8 arrays
            emit(f'rice:noise{int(noise)}:pack_device', 'rice bundle encode: one single-pass launch for lowres + 7 maps',
                 raw + b_r.numel(), t_enc_dev)
            emit(f'rice:noise{int(noise)}:unpack_device', 'rice bundle decode: one launch for lowres + 7 maps',
                 raw + b_r.numel(), t_dec_dev)
            # the file pipeline on the device, no host synchronisation: compress = the fused encode +
            # the bundle encode of its outputs, decompress = the bundle decode + the fused decode
            # (algorithmic bytes: the codec's read + write and the bundle stage's read + write)
            coder = _nd.NATURAL_CODER[tiles.dtype]
            lo3, maps3, dims3 = _nd._alloc_encoded(tiles, coder, 3)
            rec3 = torch.empty_like(tiles)
            ws3 = torch.empty(max(1, _nd.workspace_bytes(tiles, pred, 3)), dtype=torch.uint8, device='cuda')
            t_cmp = gpu_time(lambda: (_nd.fused_encode_into(tiles, pred, coder, lo3, maps3, 3, workspace=ws3),
                                      kpk._rice_encode_launch((lo3, *maps3), dims3)), args.reps)
            t_dcm = gpu_time(lambda: (kpk._rice_decode_launch(b_r, hb),
                                      _nd.fused_decode_into(lo, maps, dims, pred, coder, rec3, 3, workspace=ws3)), args.reps)
            emit(f'rice:noise{int(noise)}:compress_device', 'fused encode + rice bundle encode (device, no sync)',
                 3 * raw + b_r.numel(), t_cmp)
            emit(f'rice:noise{int(noise)}:decompress_device', 'rice bundle decode + fused decode (device, no sync)',
                 3 * raw + b_r.numel(), t_dcm)
            del lo3, maps3, rec3, ws3
            del tiles, lo, maps, maps2, lo2, b_r, b_p, vol512, res, cnt
        del field

    # the file path end to end (the user's view of compress / decompress):
    # numpy C3 volume -> container.compress -> file -> container.decompress -> numpy, host-inclusive
    # wall time (H2D, device pipeline, device CRC-32, D2H through pinned staging, file write / read),
    # with the split of the last call; structured volume (smooth field + N(0, 4^2) noise)
    if not want or 'file' in want:
        import tempfile
        zz, yy, xx = torch.meshgrid(*[torch.arange(512, device='cuda', dtype=torch.float32)] * 3, indexing='ij')
        field = torch.sin(xx / 41.0) * torch.cos(yy / 29.0) + torch.sin(zz / 53.0 + xx / 97.0)
        field = 4000 + 9000 * (field - field.min()) / (field.max() - field.min())
        del zz, yy, xx
        gen = torch.Generator(device='cuda').manual_seed(0)
        v = (field + 4.0 * torch.randn(field.shape, device='cuda', generator=gen)).round().clamp(0, 65535)
        del field
        host = v.to(torch.int32).to(torch.uint16).view(8, 64, 8, 64, 8, 64).permute(0, 2, 4, 1, 3, 5) \
            .reshape(512, 64, 64, 64, 1).contiguous().cpu().numpy()
        del v
        pred = kom.MeanPredictor(0, 3)
        with tempfile.TemporaryDirectory() as td:
            path = os.path.join(td, 'c3.kmp')
            for levels in (1, 'auto'):
                kom.container.compress(path, host, pred, levels=levels)
                assert np.array_equal(kom.container.decompress(path), host)
                tc, td_ = [], []
                splits_c, splits_d = [], []
                for _ in range(max(3, args.reps // 2)):
                    t = time.perf_counter()
                    info = kom.container.compress(path, host, pred, levels=levels)
                    tc.append(time.perf_counter() - t)
                    splits_c.append(dict(kom.container.last_timing))
                    t = time.perf_counter()
                    back = kom.container.decompress(path)  # kept: freeing the 256 MiB result is the caller's
                    td_.append(time.perf_counter() - t)
                    splits_d.append(dict(kom.container.last_timing))
                    del back
                tcm, tdm = float(np.median(tc)), float(np.median(td_))
                # the split of the median repetition, and the wall time it leaves outside its parts
                split_c = dict(splits_c[int(np.argsort(tc)[len(tc) // 2])], wall=tcm)
                split_d = dict(splits_d[int(np.argsort(td_)[len(td_) // 2])], wall=tdm)
                tag = f'file_l{levels}'
                for name, tm, split in (('compress', tcm, split_c), ('decompress', tdm, split_d)):
                    print(json.dumps({'row': f'{tag}:{name}', 'what': f'numpy 512^3 u16 (512 x 64^3) -> file -> numpy, '
                                      f'levels={levels}, MeanPredictor(0), host-inclusive',
                                      'GBps_raw': round(raw_v / tm / 1e9, 2), 'ms': round(tm * 1e3, 2),
                                      'ratio': round(info['ratio'], 3), 'file_bytes': info['bytes'],
                                      'split_ms': {k: round(v * 1e3, 2) for k, v in split.items()}}), flush=True)

    # geometry primitives (volume/utils.py) on the C3 tile batch
    if not want or 'primitives' in want:
        hp, _ = _nd.d_pad_highres(vol, 3)                       # [512, 65^3]
        lowres = _nd.d_lowres_from_highres(hp, 3)
        gt_maps = _nd.d_maps_from_highres(hp, 3)
        n_hp = hp.numel() * 2
        emit('pad_highres', 'reflect pad 64^3 -> 65^3', raw_v + n_hp, gpu_time(lambda: _nd.d_pad_highres(vol, 3), args.reps))
        emit('lowres_from_highres', 'x[:, ::2, ::2, ::2]', lowres.numel() * 4,
             gpu_time(lambda: _nd.d_lowres_from_highres(hp, 3), args.reps))
        emit('maps_from_highres', '7 parity-class gathers', n_hp - lowres.numel() * 2 + sum(m.numel() * 2 for m in gt_maps),
             gpu_time(lambda: _nd.d_maps_from_highres(hp, 3), args.reps))
        emit('highres_from_lowres_and_maps', '8-way interleave', 2 * n_hp,
             gpu_time(lambda: _nd.d_highres_from_lowres_and_maps(lowres, gt_maps, 3), args.reps))
        feats = _nd.d_features_from_lowres(lowres, 0, 3)
        emit('features_from_lowres', 'p=0: 8 shifted windows', lowres.numel() * 2 + feats.numel() * 2,
             gpu_time(lambda: _nd.d_features_from_lowres(lowres, 0, 3), args.reps))
        preds = feats[..., :1, :].expand(*feats.shape[:4], 19, 1).contiguous()
        mp = _nd.d_maps_from_predictions(preds, 3)
        emit('maps_from_predictions', 'u16 predictions, 19-way f32-order aggregation', preds.numel() * 2 + sum(m.numel() * 2 for m in mp),
             gpu_time(lambda: _nd.d_maps_from_predictions(preds, 3), args.reps))
        pf = preds.to(torch.float32)
        mpf = _nd.d_maps_from_predictions(pf, 3)
        emit('maps_from_predictions_f32', 'f32 predictions (a network output) -> f32 maps',
             pf.numel() * 4 + sum(m.numel() * 4 for m in mpf), gpu_time(lambda: _nd.d_maps_from_predictions(pf, 3), args.reps))
        del pf, mpf
        volume = vol.view(8, 8, 8, 64, 64, 64).permute(0, 3, 1, 4, 2, 5).reshape(512, 512, 512, 1)
        emit('tiles:split', '512^3 volume -> 512 x 64^3', 2 * raw_v,
             gpu_time(lambda: kom.tiles.volume_to_tiles(volume, 64), args.reps))
        emit('tiles:assemble', '512 x 64^3 -> 512^3 volume', 2 * raw_v,
             gpu_time(lambda: kom.tiles.tiles_to_volume(vol, (512, 512, 512)), args.reps))
        a, b2 = vol.view(-1), torch.empty_like(vol).view(-1)
        emit('code_u16', 'mod-2^16 coder, flat', 3 * raw_v,
             gpu_time(lambda: _nd.d_code(0, kom._lib.CODER_U16, a, b2), args.reps))


if __name__ == '__main__':
    main()
