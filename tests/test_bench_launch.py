"""bench.py's multi-GPU launcher (CPU): ``python bench.py --gpus N`` must start N ranks itself when no
external launcher set WORLD_SIZE, and refuse a launcher whose rank count differs from --gpus."""

import os
import subprocess
import sys
import textwrap

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import bench  # noqa: E402


def test_check_world_without_launcher():
    assert bench.check_world(1, {}) is False
    assert bench.check_world(2, {}) is True
    assert bench.check_world(8, {}) is True
    with pytest.raises(SystemExit):
        bench.check_world(0, {})


def test_check_world_under_launcher():
    assert bench.check_world(2, {'WORLD_SIZE': '2'}) is False
    assert bench.check_world(1, {'WORLD_SIZE': '1'}) is False
    with pytest.raises(SystemExit, match='WORLD_SIZE=4'):
        bench.check_world(8, {'WORLD_SIZE': '4'})
    with pytest.raises(SystemExit):
        bench.check_world(1, {'WORLD_SIZE': '2'})


def test_launch_command_shape():
    cmd = bench.launch_command(4, 12345, ['--gpus', '4', '--steps', '3'])
    assert cmd[:3] == [sys.executable, '-m', 'torch.distributed.run']
    assert '--nproc-per-node=4' in cmd and '--nnodes=1' in cmd
    assert cmd[cmd.index('--master-addr') + 1] == '127.0.0.1'
    assert cmd[cmd.index('--master-port') + 1] == '12345'
    assert cmd[-5:] == [os.path.abspath(bench.__file__), '--gpus', '4', '--steps', '3']


def test_launch_command_starts_n_gloo_ranks(tmp_path):
    """The command bench.maybe_launch runs really starts N ranks that rendezvous on 127.0.0.1 and
    see world size N (a stand-in script with the same argv, gloo on CPU)."""
    script = tmp_path / 'rank.py'
    script.write_text(textwrap.dedent('''
        import os, sys, torch, torch.distributed as dist
        dist.init_process_group('gloo')
        t = torch.ones(1)
        dist.all_reduce(t)
        print(f"rank={dist.get_rank()} world={dist.get_world_size()} sum={int(t.item())} argv={sys.argv[1:]}", flush=True)
        dist.destroy_process_group()
    '''))
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    env['OMP_NUM_THREADS'] = '1'
    cmd = bench.launch_command(2, bench.free_port(), ['--gpus', '2'], script=str(script))
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = sorted(l for l in r.stdout.splitlines() if l.startswith('rank='))
    assert lines == ["rank=0 world=2 sum=2 argv=['--gpus', '2']", "rank=1 world=2 sum=2 argv=['--gpus', '2']"]


def test_rank_failure_propagates(tmp_path):
    script = tmp_path / 'fail.py'
    script.write_text('import sys; sys.exit(3)\n')
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    r = subprocess.run(bench.launch_command(2, bench.free_port(), [], script=str(script)), env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
