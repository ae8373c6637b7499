"""Multi-process (gloo, world_size 2) tests of the distributed engines on CPU."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def run_workers(script, *args, nproc=2, timeout=300):
    env = dict(os.environ)
    env['CUDA_VISIBLE_DEVICES'] = ''
    env['HIP_VISIBLE_DEVICES'] = ''
    env['PYTHONPATH'] = ROOT
    env['OMP_NUM_THREADS'] = '1'
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={nproc}',
           '--master-addr=127.0.0.1', f'--master-port={_port()}', os.path.join(ROOT, 'tests', 'dist', script), *args]
    r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-4000:]
    return r.stdout


@pytest.mark.parametrize("mode", ['dp', 'os', 'os_g', 'p_g_os'])
def test_dp_and_sharding_match_single_process(mode):
    out = run_workers('worker_dp_sharding.py', mode)
    assert out.count(f'{mode} OK') == 2


@pytest.mark.parametrize("mode", ['tp', 'sp', 'pp'])
def test_hybrid_parallel_matches_single_device(mode):
    out = run_workers('worker_hybrid.py', mode)
    assert out.count(f'{mode} OK') == 2, out[-3000:]


@pytest.mark.parametrize("mode", ['os_g', 'p_g_os'])
def test_gpt_sharding_matches_single_process(mode):
    out = run_workers('worker_gpt_sharding.py', mode)
    assert out.count(f"gpt {mode} OK") == 2, out[-3000:]
