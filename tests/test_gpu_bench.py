"""bench.py end to end on the GPU box: the one-GPU line carries the contract's keys, and
``bench.py --gpus 2`` (no external launcher) starts two ranks itself -- rehearsed with gloo, the
ranks sharing the one GPU -- and reports the world size the process group saw."""

import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR',
                                                            'MASTER_PORT')}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


def test_bench_one_gpu_line():
    line = _run(['--steps', '3', '--warmup', '1', '--no-e2e', '--no-cpu-baseline'])
    for key in ('metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step', 'higher_is_better',
                'scaling', 'vs_baseline', 'dtype', 'data', 'config', 'roofline'):
        assert key in line, key
    assert line['n_gpus'] == 1 and line['dist']['world_size_seen'] == 1
    assert line['value'] > 0 and 0 < line['roofline']['frac'] < 1
    assert line['config']['workload'].startswith('512^3 uint16 volume as 512 tiles of 64^3')


def test_bench_gpus2_launches_two_ranks():
    line = _run(['--gpus', '2', '--steps', '2', '--warmup', '1', '--no-e2e'], {'KMP_BENCH_BACKEND': 'gloo'})
    assert line['n_gpus'] == 2
    assert line['dist']['world_size_seen'] == 2 and line['dist']['backend'] == 'gloo'
    assert line['config']['global_batch'] == 1024
    assert line['c4']['tiles_per_rank'] == 256
    assert line['cpu_baseline'] is None  # rank 0 at N = 1 only
