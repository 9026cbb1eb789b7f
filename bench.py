#!/usr/bin/env python3
"""Benchmark: encode+decode GB/s (device-resident) on BASELINE.json's metric workload.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload volume|image] [--padding P]

One step = one fused encode pass + one fused decode pass over the whole batch (volume: the
512^3 uint16 volume as 512 tiles of 64^3, BASELINE config C3; image: 1024 tiles of 256^2
uint8, config C2), inputs resident in HBM.  Multi-GPU (torchrun, one rank per GPU): every rank
codes its own 512-tile volume -- tiles are independent, so the path shards with no data-path
collective ("scaling": "weak"); the C4 reassembly all-gather is timed separately and reported
under "c4_reassembly", never in "value".  Rank 0 prints ONE JSON line.
"""

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)

WORKLOADS = {
    'volume': dict(ndim=3, shape=(512, 64, 64, 64, 1), dtype=np.uint16,
                   metric='encode+decode GB/s/GPU (device-resident), 512³ uint16 volume tiled 64³',
                   name='512^3 uint16 volume as 512 tiles of 64^3 (BASELINE config C3)'),
    'image': dict(ndim=2, shape=(1024, 256, 256, 1), dtype=np.uint8,
                  metric='encode+decode GB/s/GPU (device-resident), 1024 x 256² uint8 image tiles',
                  name='1024 uint8 images of 256^2 (BASELINE config C2)'),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--workload', choices=sorted(WORKLOADS), default='volume')
    ap.add_argument('--padding', type=int, default=0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument("--graph", action="store_true", help="replay each direction from a hipGraph instead of eager ctypes launches")
    ap.add_argument('--cpu-tiles', type=int, default=0, help='tiles in the CPU baseline sample (0 = all)')
    return ap.parse_args()


def synthetic(spec, seed):
    # default_rng(seed).integers over the dtype's full range
    info = np.iinfo(spec['dtype'])
    rng = np.random.default_rng(seed)
    return rng.integers(0, int(info.max) + 1, size=spec['shape'], dtype=np.int64).astype(spec['dtype'])


def cpu_baseline(spec, host, padding, ntiles):
    """The oracle (numpy op-for-op restatement of the reference's JAX path, 1 thread) on a
    bounded sample of the same workload: 1 warm-up on 4 tiles, then the median of 2 timed
    encode+decode rounds over ``ntiles`` tiles."""
    from oracle import volume as OV, image as OI, predictors as OP
    ns = OV if spec['ndim'] == 3 else OI
    enc, dec = (ns.encode_values_uint16, ns.decode_values_uint16) if spec['dtype'] == np.uint16 else \
               (ns.encode_values_uint8, ns.decode_values_uint8)
    pf = OP.mean_predictions_fn(padding, spec['ndim'])
    sample = host[:ntiles]

    def rnd(x):
        lo, (maps, dims) = ns.encode(pf, enc, x, padding=padding)
        return ns.decode(pf, dec, lo, (maps, dims), padding=padding)

    rnd(host[:4])
    times = []
    for _ in range(2):
        t = time.perf_counter()
        out = rnd(sample)
        times.append(time.perf_counter() - t)
    assert np.array_equal(out, sample), 'oracle round trip failed'
    t = float(np.median(times))
    return {'value': round(sample.nbytes / t / 1e9, 4), 'unit': 'GB/s', 'cores': 1, 'kind': 'port',
            'sample': f'{ntiles} of {host.shape[0]} tiles, numpy restatement of the reference path '
                      f'(oracle/, materialised features/predictions, 1 thread; host has '
                      f'{len(os.sched_getaffinity(0))} cores), median of 2 after warm-up, {t:.2f} s/round'}


def load_traffic(workload, padding, kernel):
    """HBM bytes per launch of ``kernel`` from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, collected by separate --pmc FETCH_SIZE / WRITE_SIZE passes of this
    same command), or None when no such measurement exists."""
    path = os.path.join(HERE, 'profiles', 'pmc_traffic.json')
    if not os.path.exists(path):
        return None
    with open(path) as f:
        entry = json.load(f).get(f'{workload}_p{padding}', {}).get(kernel)
    return entry['hbm_bytes'] if entry else None


def main():
    args = parse()
    spec = WORKLOADS[args.workload]
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    else:
        dist = None
        torch.cuda.set_device(0)

    import kompressor_amd as kom
    from kompressor_amd import _nd
    ndim = spec['ndim']
    ns = kom.volume if ndim == 3 else kom.image
    predictor = kom.MeanPredictor(args.padding, ndim)
    coder = _nd.NATURAL_CODER[torch.uint16 if spec['dtype'] == np.uint16 else torch.uint8]

    host = synthetic(spec, seed=rank)
    hi = torch.from_numpy(host).cuda()
    lowres, maps, dims = _nd._alloc_encoded(hi, coder, ndim)
    rec = torch.empty_like(hi)
    ws = torch.empty(max(1, _nd.workspace_bytes(hi, predictor, ndim)), dtype=torch.uint8, device='cuda')

    def encode():
        _nd.fused_encode_into(hi, predictor, coder, lowres, maps, ndim, workspace=ws)

    def decode():
        _nd.fused_decode_into(lowres, maps, dims, predictor, coder, rec, ndim, workspace=ws)

    # correctness gate before timing: lossless round trip of the whole batch
    encode()
    decode()
    torch.cuda.synchronize()
    assert torch.equal(rec, hi), 'round trip is not lossless'

    for _ in range(args.warmup):
        encode()
        decode()
    if not args.graph:
        run_enc, run_dec = encode, decode
    else:
        # one hipGraph per direction: replays the same single kernel launch without the Python /
        # ctypes launch path (measured: no gain at this size, profiles/round1/bench_graph_vs_eager.log)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            encode()
            decode()
        torch.cuda.current_stream().wait_stream(side)
        g_enc, g_dec = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_enc):
            encode()
        with torch.cuda.graph(g_dec):
            decode()
        run_enc, run_dec = g_enc.replay, g_dec.replay
        for _ in range(2):
            run_enc()
            run_dec()
        torch.cuda.synchronize()
        assert torch.equal(rec, hi), 'graph replay round trip is not lossless'
    stream = torch.cuda.current_stream()  # the stream the kernels / graphs are launched on
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for e0, e1, e2 in ev:
        e0.record(stream)
        run_enc()
        e1.record(stream)
        run_dec()
        e2.record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t_enc = float(np.mean([a.elapsed_time(b) for a, b, _ in ev])) / 1e3
    t_dec = float(np.mean([b.elapsed_time(c) for _, b, c in ev])) / 1e3
    if dist:
        tt = torch.tensor([elapsed, t_enc, t_dec], dtype=torch.float64, device='cuda')
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, t_enc, t_dec = tt.tolist()

    raw = hi.numel() * hi.element_size()           # raw highres bytes per rank per step
    value = raw * world * args.steps / elapsed / 1e9
    ms_per_step = elapsed / args.steps * 1e3
    # algorithmic HBM bytes per launch: read + write of the raw volume
    algo = 2 * raw
    dominant, t_dom = ('encode', t_enc) if t_enc >= t_dec else ('decode', t_dec)
    achieved = algo / t_dom / 1e9
    traffic = load_traffic(args.workload, args.padding, dominant)

    # C4: shard one volume's tiles over the ranks, code them, all-gather the decoded tiles
    c4 = None
    if dist:
        per = spec['shape'][0] // world
        shard = hi[:per].contiguous()
        lo_s, maps_s, dims_s = _nd._alloc_encoded(shard, coder, ndim)
        rec_s = torch.empty_like(shard)
        full = torch.empty((per * world, *shard.shape[1:]), dtype=torch.int16, device='cuda')
        times = []
        for i in range(6):
            dist.barrier()
            torch.cuda.synchronize()
            t = time.perf_counter()
            _nd.fused_encode_into(shard, predictor, coder, lo_s, maps_s, ndim, workspace=ws)
            _nd.fused_decode_into(lo_s, maps_s, dims_s, predictor, coder, rec_s, ndim, workspace=ws)
            dist.all_gather_into_tensor(full, rec_s.view(torch.int16))
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t)
        tt = torch.tensor([float(np.median(times[1:]))], dtype=torch.float64, device='cuda')
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        c4 = {'tiles_per_rank': per, 'ms_codec_plus_allgather': round(tt.item() * 1e3, 4),
              'volume_GBps': round(raw / tt.item() / 1e9, 2), 'collective': 'all_gather_into_tensor (RCCL)'}

    base = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        base = cpu_baseline(spec, host, args.padding, args.cpu_tiles or spec['shape'][0])

    if rank == 0:
        line = {
            'metric': spec['metric'], 'value': round(value, 3), 'unit': 'GB/s', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(ms_per_step, 5),
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
            'dtype': 'u16' if spec['dtype'] == np.uint16 else 'u8', 'data': 'synthetic (default_rng uniform)',
            'config': {'workload': spec['name'], 'global_batch': spec['shape'][0] * world,
                       'tile': list(spec['shape'][1:-1]), 'predictor': f'MeanPredictor(padding={args.padding})',
                       'parallelism': f'tiles sharded, dp{world}' if world > 1 else 'single GPU'},
            'ms_encode': round(t_enc * 1e3, 5), 'ms_decode': round(t_dec * 1e3, 5),
            'launch': 'hipGraph replay (one graph per direction)' if args.graph else 'eager (one ctypes launch per direction)',
            'roofline': {'bound': 'hbm', 'kernel': f'fast3d_kernel {dominant}' if ndim == 3 else f'{dominant}',
                         'achieved': round(achieved, 2), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': round(achieved / HBM_PEAK_GBS, 4),
                         'traffic': traffic, 'algorithmic_bytes_per_launch': algo},
            'cpu_baseline': base,
        }
        if c4:
            line['c4_reassembly'] = c4
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
