#!/usr/bin/env python3
"""Benchmark: encode+decode GB/s (device-resident) on BASELINE.json's metric workload.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload volume|image] [--padding P]

One step = one fused encode pass + one fused decode pass over the whole batch (volume: the
512^3 uint16 volume as 512 tiles of 64^3, BASELINE config C3; image: 1024 tiles of 256^2
uint8, config C2), inputs resident in HBM.  Multi-GPU (torchrun, one rank per GPU): every rank
codes its own 512-tile volume -- tiles are independent, so the path shards with no data-path
collective ("scaling": "weak"; ``value`` = bytes coded by all ranks / wall time, the whole-job
aggregate, ``value_per_gpu`` = value / N).  Config C4 proper -- ONE volume, 512/N tiles per rank,
then the RCCL all-gather that reassembles it -- is measured beside it under "c4" (codec and
all-gather timed separately), never in ``value``.  Rank 0 prints ONE JSON line.
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
    # C5: 2048^3 float32 = 4096 chunks of 128^3 over 8 GPUs -> 512 chunks (4 GiB) per GPU,
    # host-resident (pinned): the fused kernels read / write the pinned host arrays over the link
    'stream': dict(ndim=3, shape=(512, 128, 128, 128, 1), dtype=np.float32,
                   metric='encode+decode GB/s/GPU (pinned host -> GPU -> host), 2048³ float32 as 128³ chunks',
                   name='2048^3 float32 streamed as 128^3 chunks, 512 chunks per GPU (BASELINE config C5)'),
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
    ap.add_argument('--cpu-tiles', type=int, default=0,
                    help='tiles in the 1-thread numpy CPU sample (0 = 64 volume tiles / 256 images)')
    ap.add_argument('--e2e-chunk', type=int, default=32, help='tiles per H2D/D2H copy in the end-to-end leg')
    ap.add_argument('--no-e2e', action='store_true', help='skip the pinned-host end-to-end leg')
    ap.add_argument('--stream-tiles', type=int, default=0, help='stream workload: chunks per GPU (0 = 512)')
    return ap.parse_args()


def synthetic(spec, seed):
    # default_rng(seed).integers over the dtype's full range
    if spec['dtype'] == np.float32:
        return np.random.default_rng(seed).standard_normal(spec['shape'], dtype=np.float32)
    info = np.iinfo(spec['dtype'])
    rng = np.random.default_rng(seed)
    return rng.integers(0, int(info.max) + 1, size=spec['shape'], dtype=np.int64).astype(spec['dtype'])


def _median_rate(fn, nbytes, reps=5):
    """1 warm-up, then the median of ``reps`` timed runs of ``fn`` -> (GB/s, median seconds)."""
    fn()
    times = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        times.append(time.perf_counter() - t)
    t = float(np.median(times))
    return nbytes / t / 1e9, t


def host_cores():
    """The host cores this process may run on: the affinity mask, capped by a cgroup CPU quota
    when one is set (cgroup v2 ``cpu.max``, else v1 ``cpu.cfs_quota_us``).  Returns (cores, how)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        if q != 'max':
            quota = -(-int(q) // int(per))
    except (OSError, ValueError):
        try:
            q = int(open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us').read())
            per = int(open('/sys/fs/cgroup/cpu/cpu.cfs_period_us').read())
            if q > 0:
                quota = -(-q // per)
        except (OSError, ValueError):
            pass
    if quota is not None and quota < aff:
        return quota, f'cgroup CPU quota {quota} of {aff} cores in the affinity mask'
    return aff, f'the affinity mask ({aff} cores, no smaller cgroup CPU quota)'


def cpu_baseline(spec, host, padding, ntiles_numpy=0, ntiles_torch=0):
    """The reference path on the host cores, on a bounded sample of the same workload
    (BASELINE.md §2): 1 warm-up + the median of 5 encode+decode rounds of
      * the multithreaded torch-CPU restatement (oracle/torch_cpu.py: the reference's op sequence
        with its materialised features / predictions, every op a torch CPU kernel on
        torch.get_num_threads() threads) -- the headline ``value``;
      * the 1-thread numpy op-for-op restatement (oracle/volume.py, oracle/image.py) beside it.
    Both round trips are checked lossless."""
    from oracle import volume as OV, image as OI, predictors as OP, torch_cpu as TC
    ndim = spec['ndim']
    ns = OV if ndim == 3 else OI
    enc, dec = (ns.encode_values_uint16, ns.decode_values_uint16) if spec['dtype'] == np.uint16 else \
               (ns.encode_values_uint8, ns.decode_values_uint8)
    pf = OP.mean_predictions_fn(padding, ndim)
    n = host.shape[0]
    nn = min(n, ntiles_numpy or (64 if ndim == 3 else 256))
    nt = min(n, ntiles_torch or n)
    out = {}

    def numpy_round():
        lo, (maps, dims) = ns.encode(pf, enc, host[:nn], padding=padding)
        out['np'] = ns.decode(pf, dec, lo, (maps, dims), padding=padding)

    def torch_round():
        lo, e = TC.encode(host[:nt], padding, ndim)
        out['torch'] = TC.decode(lo, e, padding, ndim)

    threads, how = host_cores()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        r_t, t_t = _median_rate(torch_round, host[:nt].nbytes)
    finally:
        torch.set_num_threads(prev)
    assert np.array_equal(out['torch'], host[:nt]), 'torch-CPU round trip failed'
    r_n, t_n = _median_rate(numpy_round, host[:nn].nbytes)
    assert np.array_equal(out['np'], host[:nn]), 'oracle round trip failed'
    unit = 'tiles' if ndim == 3 else 'images'
    return {'value': round(r_t, 4), 'unit': 'GB/s', 'cores': threads, 'kind': 'port',
            'sample': f'{nt} of {n} {unit}: torch-CPU restatement of the reference path (oracle/torch_cpu.py, '
                      f'materialised features / predictions like the JAX path) on {threads} threads '
                      f'(every host core this process may use: {how}), '
                      f'1 warm-up + median of 5 encode+decode rounds, {t_t:.3f} s/round',
            'single_thread_numpy': {'value': round(r_n, 4), 'unit': 'GB/s', 'cores': 1, 'kind': 'port',
                                    'sample': f'{nn} of {n} {unit}: numpy op-for-op restatement (oracle/), '
                                              f'1 thread, 1 warm-up + median of 5, {t_n:.3f} s/round'}}


def e2e_leg(kom, host, predictor, ndim, chunk, reps=3):
    """Host-resident rate: pinned host tiles in, pinned host outputs out, per direction
    (kompressor_amd.stream.TileStream: zero-copy fused kernels by default, KMP_STREAM_COPY=1 a
    3-stream H2D / kernel / D2H pipeline).  Median of ``reps`` after one warm-up."""
    src = kom.stream.pinned(host.shape, torch.from_numpy(host[:0]).dtype)
    src.copy_(torch.from_numpy(host))
    ts = kom.stream.TileStream(predictor, host.shape[1:], src.dtype, chunk, 3, ndim)
    lo, maps = ts.alloc_encoded(host.shape[0])
    out = kom.stream.pinned(host.shape, src.dtype)
    te, td = [], []
    for i in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ts.encode(src, lo, maps)
        ts.synchronize()
        t1 = time.perf_counter()
        ts.decode(lo, maps, out)
        ts.synchronize()
        t2 = time.perf_counter()
        if i:
            te.append(t1 - t0)
            td.append(t2 - t1)
    assert torch.equal(out.view(torch.uint8), src.view(torch.uint8)), 'end-to-end round trip is not lossless'
    te, td = float(np.median(te)), float(np.median(td))
    raw = src.numel() * src.element_size()
    return {'GBps': round(raw / (te + td) / 1e9, 3), 'ms_encode': round(te * 1e3, 3), 'ms_decode': round(td * 1e3, 3),
            'mode': 'zero-copy (kernels read / write pinned host memory over the link)' if ts.zero_copy
                    else f'copy pipeline ({chunk}-tile chunks, 3 streams)',
            'host_memory': 'pinned',
            'note': 'raw bytes / (t_enc + t_dec), each direction timed from pinned host input to pinned host output'}


def kernel_name(ndim, padding, direction='encode', u8=False):
    # the one-pass kernel the C layer dispatches for this workload (kmp_codec_*.hip)
    if ndim == 3:
        return 'wave3d_plane_kernel' if padding == 0 else 'fast3d_kernel'
    if padding == 0:
        return 'wave2d_u8_kernel' if (u8 and direction == 'decode') else 'wave2d_kernel'
    return 'wave2dp_kernel'


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


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def launch_command(n, port, argv, script=None):
    """The command that starts ``n`` rank processes of this script (one per GPU) with the same
    arguments: torch.distributed.run on one node, rendezvous on 127.0.0.1."""
    return [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
            '--master-addr', '127.0.0.1', '--master-port', str(port),
            script or os.path.abspath(__file__), *argv]


def check_world(gpus, env):
    """Under a launcher (``WORLD_SIZE`` set) the rank count must equal ``--gpus``; returns True when
    this process must launch the ranks itself (``--gpus N > 1`` and no launcher)."""
    ws = env.get('WORLD_SIZE')
    if ws is not None:
        if int(ws) != gpus:
            raise SystemExit(f'bench.py: --gpus {gpus} but the launcher started WORLD_SIZE={ws} ranks')
        return False
    if gpus < 1:
        raise SystemExit(f'bench.py: --gpus must be >= 1, got {gpus}')
    return gpus > 1


def maybe_launch(args):
    """``python bench.py --gpus N`` with N > 1 and no external launcher: start N ranks here, before
    this process makes any GPU call (``torch.cuda.device_count`` does not initialise the device on
    this image), and return their exit status; None when this process is a rank itself."""
    if not check_world(args.gpus, os.environ):
        return None
    backend = os.environ.get('KMP_BENCH_BACKEND', 'nccl')
    have = torch.cuda.device_count()
    if backend == 'nccl' and have < args.gpus:
        raise SystemExit(f'bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs for RCCL, '
                         f'{have} visible (KMP_BENCH_BACKEND=gloo rehearses N ranks on fewer)')
    import subprocess
    return subprocess.call(launch_command(args.gpus, free_port(), sys.argv[1:]))


def init_dist():
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        import torch.distributed as dist
        # one process per GPU over RCCL; KMP_BENCH_BACKEND=gloo rehearses the N > 1 logic with
        # every rank on the devices one box has (ranks share a GPU when there are fewer GPUs)
        backend = os.environ.get('KMP_BENCH_BACKEND', 'nccl')
        dev_id = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev_id)
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', dev_id))
        else:
            dist.init_process_group(backend)
        seen = dist.get_world_size()
        assert seen == world, f'process group has {seen} ranks, WORLD_SIZE is {world}'
    else:
        dist = None
        torch.cuda.set_device(0)
    return world, rank, dist


def dist_info(dist, world):
    """What the job actually ran on: the rank count the process group reports after init."""
    if not dist:
        return {'world_size_seen': 1, 'backend': None, 'launcher': 'none (single process)'}
    return {'world_size_seen': dist.get_world_size(), 'backend': dist.get_backend(),
            'launcher': 'torch.distributed.run (one rank per GPU)'}


def timed_steps(run_enc, run_dec, steps, dist):
    """EXACTLY ``steps`` (encode, decode) pairs bracketed by barrier + synchronize on both sides;
    wall seconds, max over ranks.  Nothing else is enqueued inside the region."""
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        run_enc()
        run_dec()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device='cuda')
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = tt.item()
    return elapsed


_SLEEP_RATE = []


def _sleep_cycles(seconds):
    """torch.cuda._sleep cycles for ``seconds`` of device time (rate calibrated once with events)."""
    if not _SLEEP_RATE:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        torch.cuda._sleep(1_000_000)
        e1.record()
        torch.cuda.synchronize()
        _SLEEP_RATE.append(1_000_000 / max(e0.elapsed_time(e1) / 1e3, 1e-6))  # cycles per second
    return int(seconds * _SLEEP_RATE[0]) + 1


def direction_times(run_enc, run_dec, n, dist):
    """Average kernel duration per direction from HIP events on the launch stream, over ``n``
    encode / decode pairs alternating as the timed loop runs them (an event between every two
    launches, so each interval is one kernel plus its launch boundary, in the cache state of the
    timed region); max over ranks.  This is what ``roofline.achieved`` divides by and what the
    committed rocprofv3 kernel statistics must agree with."""
    stream = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * n + 1)]
    torch.cuda.synchronize()
    # keep the GPU busy (untimed) while the host enqueues all 2n launches, so the events time the
    # kernels back to back on the device and not the host's launch rate (an eager launch costs
    # ~20-45 us of Python / ctypes, as long as a C2 kernel)
    torch.cuda._sleep(_sleep_cycles(2 * n * 100e-6))
    ev[0].record(stream)
    for i in range(n):
        run_enc()
        ev[2 * i + 1].record(stream)
        run_dec()
        ev[2 * i + 2].record(stream)
    torch.cuda.synchronize()
    t_enc = sum(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(n)) / n / 1e3
    t_dec = sum(ev[2 * i + 1].elapsed_time(ev[2 * i + 2]) for i in range(n)) / n / 1e3
    if dist:
        tt = torch.tensor([t_enc, t_dec], dtype=torch.float64, device='cuda')
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_enc, t_dec = tt.tolist()
    return t_enc, t_dec


def c4_strong(kom, hi, predictor, ndim, dist, world, ws, reps=10):
    """BASELINE config C4 as SURVEY.md §8d defines it: ONE 512^3 volume (rank 0's, broadcast),
    its 512 tiles sharded 512/N per rank (kompressor_amd.shard), each rank codes its shard, then
    one RCCL all-gather reassembles the decoded volume on every rank.  Codec and all-gather are
    timed separately (barrier + synchronize around each, max over ranks, median of ``reps``);
    reported beside ``value``, never in it."""
    from kompressor_amd import _nd
    hi = hi.clone()
    dist.broadcast(hi.view(torch.uint8), 0)   # every rank holds the same volume (rank 0's)
    n = hi.shape[0]
    shard = kom.shard.local_shard(hi).contiguous()
    coder = _nd.NATURAL_CODER[hi.dtype]
    lo_s, maps_s, dims_s = _nd._alloc_encoded(shard, coder, ndim)
    rec_s = torch.empty_like(shard)

    def codec():
        _nd.fused_encode_into(shard, predictor, coder, lo_s, maps_s, ndim, workspace=ws)
        _nd.fused_decode_into(lo_s, maps_s, dims_s, predictor, coder, rec_s, ndim, workspace=ws)

    def timed(fn):
        ts = []
        for i in range(reps + 2):
            dist.barrier()
            torch.cuda.synchronize()
            t = time.perf_counter()
            r = fn()
            torch.cuda.synchronize()
            if i >= 2:
                ts.append(time.perf_counter() - t)
        tt = torch.tensor([float(np.median(ts))], dtype=torch.float64, device='cuda')
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return tt.item(), r

    t_codec, _ = timed(codec)
    t_ag, full = timed(lambda: kom.shard.all_gather_tiles(rec_s, n))
    assert torch.equal(full, hi), 'C4 reassembled volume differs from the input'
    raw = hi.numel() * hi.element_size()
    recv = raw - shard.numel() * shard.element_size()
    return {'tiles_per_rank': int(shard.shape[0]), 'ms_codec': round(t_codec * 1e3, 4),
            'ms_allgather': round(t_ag * 1e3, 4),
            'volume_GBps_codec': round(raw / t_codec / 1e9, 2),
            'volume_GBps_with_reassembly': round(raw / (t_codec + t_ag) / 1e9, 2),
            'allgather_GBps_received_per_rank': round(recv / t_ag / 1e9, 2),
            'scaling': 'strong (one 512^3 volume split over the ranks)',
            'collective': ('all_gather_into_tensor (RCCL over xGMI) of per-rank decoded tile slabs'
                           if dist.get_backend() == 'nccl' else f'all_gather ({dist.get_backend()}) of per-rank decoded tile slabs')}


def main():
    args = parse()
    rc = maybe_launch(args)
    if rc is not None:
        sys.exit(rc)
    if args.workload == 'stream':
        return main_stream(args)
    spec = WORKLOADS[args.workload]
    world, rank, dist = init_dist()

    import kompressor_amd as kom
    from kompressor_amd import _nd
    ndim = spec['ndim']
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
    elapsed = timed_steps(run_enc, run_dec, args.steps, dist)
    t_enc, t_dec = direction_times(run_enc, run_dec, max(args.steps, 10), dist)

    raw = hi.numel() * hi.element_size()           # raw highres bytes per rank per step
    value = raw * world * args.steps / elapsed / 1e9
    ms_per_step = elapsed / args.steps * 1e3
    # algorithmic HBM bytes per launch: read + write of the raw volume
    algo = 2 * raw
    dominant, t_dom = ('encode', t_enc) if t_enc >= t_dec else ('decode', t_dec)
    achieved = algo / t_dom / 1e9
    traffic = load_traffic(args.workload, args.padding, dominant)

    c4 = c4_strong(kom, hi, predictor, ndim, dist, world, ws) if dist else None

    e2e = None
    if world == 1 and not args.no_e2e:
        e2e = e2e_leg(kom, host, predictor, ndim, args.e2e_chunk)

    base = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        base = cpu_baseline(spec, host, args.padding, args.cpu_tiles)

    if rank == 0:
        line = {
            'metric': spec['metric'], 'value': round(value, 3), 'unit': 'GB/s', 'n_gpus': world,
            'value_per_gpu': round(value / world, 3),
            'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(ms_per_step, 5),
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
            'dtype': 'u16' if spec['dtype'] == np.uint16 else 'u8', 'data': 'synthetic (default_rng uniform)',
            'config': {'workload': spec['name'], 'global_batch': spec['shape'][0] * world,
                       'tile': list(spec['shape'][1:-1]), 'predictor': f'MeanPredictor(padding={args.padding})',
                       'parallelism': f'tiles sharded, dp{world}' if world > 1 else 'single GPU',
                       'value_is': 'whole-job aggregate: raw highres bytes coded by all ranks / wall time '
                                   '(weak scaling: every rank codes its own full batch; value_per_gpu = value / n_gpus)'},
            'ms_encode': round(t_enc * 1e3, 5), 'ms_decode': round(t_dec * 1e3, 5),
            'dist': dist_info(dist, world),
            'launch': 'hipGraph replay (one graph per direction)' if args.graph else 'eager (one ctypes launch per direction)',
            'roofline': {'bound': 'hbm', 'kernel': f'{kernel_name(ndim, args.padding, dominant, spec["dtype"] == np.uint8)} {dominant}',
                         'achieved': round(achieved, 2), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': round(achieved / HBM_PEAK_GBS, 4),
                         'traffic': traffic, 'algorithmic_bytes_per_launch': algo},
            'cpu_baseline': base,
        }
        if e2e:
            line['e2e_host'] = e2e
        if c4:
            line['c4'] = c4
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


def main_stream(args):
    """BASELINE config C5: each GPU streams its 512 chunks of 128^3 float32 (4 GiB) from pinned
    host memory through the codec and back (kompressor_amd.stream.TileStream, 3 streams).  One
    step = the encode stream + the decode stream of all the rank's chunks; ``value`` = raw
    bytes of all ranks / wall time.  Chunks are independent, so ranks share nothing."""
    spec = dict(WORKLOADS['stream'])
    n = args.stream_tiles or spec['shape'][0]
    spec['shape'] = (n, *spec['shape'][1:])
    world, rank, dist = init_dist()
    import kompressor_amd as kom
    from kompressor_amd import _nd
    predictor = kom.MeanPredictor(args.padding, 3)
    chunk_shape = spec['shape'][1:]
    # synthetic float32 chunks: 16 distinct random chunks tiled over the batch (the codec's cost
    # is data-independent; this keeps host generation of 4 GiB to a copy)
    seed_chunks = np.random.default_rng(rank).standard_normal((min(16, n), *chunk_shape), dtype=np.float32)
    src = kom.stream.pinned(spec['shape'], torch.float32)
    for b in range(0, n, seed_chunks.shape[0]):
        e = min(n, b + seed_chunks.shape[0])
        src[b:e].copy_(torch.from_numpy(seed_chunks[:e - b]))
    ts = kom.stream.TileStream(predictor, chunk_shape, torch.float32, 1, 3, 3)
    lo, maps = ts.alloc_encoded(n)
    out = kom.stream.pinned(spec['shape'], torch.float32)

    def step():
        ts.encode(src, lo, maps)
        ts.synchronize()
        t = time.perf_counter()
        ts.decode(lo, maps, out)
        ts.synchronize()
        return t

    step()
    assert torch.equal(out.view(torch.uint32), src.view(torch.uint32)), 'C5 round trip is not lossless'
    for _ in range(args.warmup):
        step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    t_enc = 0.0
    for _ in range(args.steps):
        t_s = time.perf_counter()
        t_mid = step()
        t_enc += t_mid - t_s
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t_dec = elapsed - t_enc
    if dist:
        tt = torch.tensor([elapsed, t_enc, t_dec], dtype=torch.float64, device='cuda')
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, t_enc, t_dec = tt.tolist()
    raw = src.numel() * 4

    # kernel roofline of the same codec device-resident (the uint32 one-pass kernel,
    # kmp_codec_wave3d32.hip) on a 64-chunk slice
    k = min(64, n)
    d_hi = src[:k].cuda().view(torch.uint32)
    coder = _nd.NATURAL_CODER[torch.uint32]
    d_lo, d_maps, d_dims = _nd._alloc_encoded(d_hi, coder, 3)
    d_rec = torch.empty_like(d_hi)
    ws = torch.empty(max(1, _nd.workspace_bytes(d_hi, predictor, 3)), dtype=torch.uint8, device='cuda')
    enc = lambda: _nd.fused_encode_into(d_hi, predictor, coder, d_lo, d_maps, 3, workspace=ws)  # noqa: E731
    dec = lambda: _nd.fused_decode_into(d_lo, d_maps, d_dims, predictor, coder, d_rec, 3, workspace=ws)  # noqa: E731
    enc()
    kname_enc = kom._lib.lib.kmp_last_launch().decode()
    dec()
    kname_dec = kom._lib.lib.kmp_last_launch().decode()
    k_enc, k_dec = direction_times(enc, dec, 5, None)
    assert torch.equal(d_rec, d_hi)
    kraw = d_hi.numel() * 4
    dominant, t_dom = ('encode', k_enc) if k_enc >= k_dec else ('decode', k_dec)
    achieved = 2 * kraw / t_dom / 1e9

    base = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the same two restatements as the C3 / C2 lines, on the uint32 bit patterns
        from oracle import volume as OV, predictors as OP, torch_cpu as TC
        host32 = src.numpy().view(np.uint32)
        pf = OP.mean_predictions_fn(args.padding, 3)
        nn, nt = min(n, 2), min(n, 8)
        out = {}

        def numpy_round():
            lo_o, enc_o = OV.encode(pf, OV.encode_values_uint32, host32[:nn], padding=args.padding)
            out['np'] = OV.decode(pf, OV.decode_values_uint32, lo_o, enc_o, padding=args.padding)

        def torch_round():
            lo_t, enc_t = TC.encode(host32[:nt], args.padding, 3)
            out['torch'] = TC.decode(lo_t, enc_t, args.padding, 3)

        threads, how = host_cores()
        prev = torch.get_num_threads()
        torch.set_num_threads(threads)
        try:
            r_t, t_t = _median_rate(torch_round, host32[:nt].nbytes)
        finally:
            torch.set_num_threads(prev)
        assert np.array_equal(out['torch'], host32[:nt])
        r_n, t_n = _median_rate(numpy_round, host32[:nn].nbytes)
        assert np.array_equal(out['np'], host32[:nn])
        base = {'value': round(r_t, 4), 'unit': 'GB/s', 'cores': threads, 'kind': 'port',
                'sample': f'{nt} of {n} chunks of 128^3: torch-CPU restatement (oracle/torch_cpu.py, uint32 '
                          f'bit-cast) on {threads} threads ({how}), 1 warm-up + median of 5, {t_t:.3f} s/round',
                'single_thread_numpy': {'value': round(r_n, 4), 'unit': 'GB/s', 'cores': 1, 'kind': 'port',
                                        'sample': f'{nn} of {n} chunks, numpy restatement (oracle/), 1 thread, '
                                                  f'1 warm-up + median of 5, {t_n:.3f} s/round'}}
    if rank == 0:
        line = {
            'metric': spec['metric'], 'value': round(raw * world * args.steps / elapsed / 1e9, 3), 'unit': 'GB/s',
            'value_per_gpu': round(raw * args.steps / elapsed / 1e9, 3),
            'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': round(elapsed / args.steps * 1e3, 3), 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': 'u32 (float32 bit-cast)', 'data': 'synthetic (standard normal float32)',
            'config': {'workload': spec['name'], 'global_batch': n * world, 'tile': list(chunk_shape[:3]),
                       'predictor': f'MeanPredictor(padding={args.padding})',
                       'mode': 'zero-copy (one fused launch per direction reads / writes pinned host memory)'
                               if ts.zero_copy else 'copy pipeline (3 streams, 1 chunk per copy)',
                       'parallelism': f'chunks sharded, dp{world}' if world > 1 else 'single GPU'},
            'ms_encode': round(t_enc / args.steps * 1e3, 3), 'ms_decode': round(t_dec / args.steps * 1e3, 3),
            'roofline': {'bound': 'hbm', 'kernel': kname_enc if dominant == 'encode' else kname_dec,
                         'achieved': round(achieved, 2), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': round(achieved / HBM_PEAK_GBS, 4), 'traffic': None,
                         'algorithmic_bytes_per_launch': 2 * kraw,
                         'device_resident_ms': {'encode': round(k_enc * 1e3, 4), 'decode': round(k_dec * 1e3, 4),
                                                'chunks': k}},
            'dist': dist_info(dist, world),
            'link': {'h2d_plus_d2h_bytes_per_step': 4 * raw,
                     'note': 'each direction moves the raw volume host->device and its coded form back'},
            'cpu_baseline': base,
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
