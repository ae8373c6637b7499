"""Process-group bootstrap (reference: python/paddle/distributed/parallel.py:945 init_parallel_env,
:644 ParallelEnv, python/paddle/distributed/spawn.py).

One process per MI355X: rank/world/local-rank come from the launcher's environment
(PADDLE_TRAINER_ID / PADDLE_TRAINERS_NUM as the reference's launcher sets them, or the
RANK / WORLD_SIZE / LOCAL_RANK of torch.distributed.run); the default backend is RCCL
("nccl") when a GPU is visible, gloo otherwise.
"""
import atexit
import datetime
import os

import torch
import torch.distributed as dist

from . import communication as C


def _env_int(*names, default=0):
    for n in names:
        v = os.environ.get(n)
        if v not in (None, ''):
            return int(v)
    return default


class ParallelEnv:
    def __init__(self):
        self._rank = _env_int('PADDLE_TRAINER_ID', 'RANK', default=0)
        self._world_size = _env_int('PADDLE_TRAINERS_NUM', 'WORLD_SIZE', default=1)
        self._local_rank = _env_int('PADDLE_LOCAL_RANK', 'LOCAL_RANK', default=self._rank)
        self._device_id = self._local_rank
        eps = os.environ.get('PADDLE_TRAINER_ENDPOINTS', '')
        self._trainer_endpoints = eps.split(',') if eps else []
        self._current_endpoint = os.environ.get('PADDLE_CURRENT_ENDPOINT', '')
        self._nrings = 1

    @property
    def rank(self):
        return self._rank

    @property
    def world_size(self):
        return self._world_size

    @property
    def local_rank(self):
        return self._local_rank

    @property
    def device_id(self):
        return self._device_id

    @property
    def device_type(self):
        return 'gpu' if torch.cuda.is_available() else 'cpu'

    @property
    def current_endpoint(self):
        return self._current_endpoint

    @property
    def trainer_endpoints(self):
        return self._trainer_endpoints

    @property
    def nrings(self):
        return self._nrings

    local_rank_ = local_rank
    nranks = world_size
    dev_id = device_id


def _destroy_at_exit():
    """Tear the process group down before interpreter teardown: a rank that exits with gloo's
    pair threads still joinable dies in std::terminate (exit status -6) after finishing its work."""
    try:
        if dist.is_initialized():
            dist.destroy_process_group()
    except Exception:  # exit path: never mask the program's own status
        pass


def init_parallel_env(backend=None, timeout_s=None):
    """Initialise the global process group (idempotent); returns the global Group."""
    env = ParallelEnv()
    if not dist.is_initialized() and env.world_size > 1:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        if 'MASTER_PORT' not in os.environ:
            ep = os.environ.get('PADDLE_TRAINER_ENDPOINTS', '').split(',')[0]
            os.environ['MASTER_PORT'] = ep.split(':')[1] if ':' in ep else '29500'
        use_gpu = torch.cuda.is_available()
        be = backend or ('nccl' if use_gpu else 'gloo')
        be = {'rccl': 'nccl', 'nccl': 'nccl', 'gloo': 'gloo', 'auto': 'nccl' if use_gpu else 'gloo'}.get(be, be)
        kw = {}
        if timeout_s:
            kw['timeout'] = datetime.timedelta(seconds=timeout_s)
        if be == 'nccl':
            torch.cuda.set_device(env.local_rank % max(torch.cuda.device_count(), 1))
            kw['device_id'] = torch.device('cuda', torch.cuda.current_device())
        dist.init_process_group(be, rank=env.rank, world_size=env.world_size, **kw)
        atexit.register(_destroy_at_exit)
        from ..core import place
        if be == 'nccl':
            place.set_device(f'gpu:{torch.cuda.current_device()}')
    C._global[0] = None
    return C._world()


def get_rank(group=None):
    return C.get_rank(group)


def get_world_size(group=None):
    return C.get_world_size(group)


def _spawn_worker(fn, rank, nprocs, args, backend, port, env_extra):
    os.environ.update({'PADDLE_TRAINER_ID': str(rank), 'RANK': str(rank), 'LOCAL_RANK': str(rank),
                       'PADDLE_TRAINERS_NUM': str(nprocs), 'WORLD_SIZE': str(nprocs), 'MASTER_ADDR': '127.0.0.1',
                       'MASTER_PORT': str(port)})
    os.environ.update(env_extra)
    fn(*args)


def spawn(func, args=(), nprocs=-1, join=True, daemon=False, **options):
    """paddle.distributed.spawn: start nprocs worker processes running func(*args)."""
    import socket
    import torch.multiprocessing as mp
    if nprocs == -1:
        nprocs = max(torch.cuda.device_count(), 1)
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    env_extra = {'HSA_ENABLE_IPC_MODE_LEGACY': os.environ.get('HSA_ENABLE_IPC_MODE_LEGACY', '0')}
    procs = []
    mpctx = mp.get_context('spawn')
    for r in range(nprocs):
        p = mpctx.Process(target=_spawn_worker, args=(func, r, nprocs, args, options.get('backend'), port, env_extra),
                          daemon=daemon)
        p.start()
        procs.append(p)
    if join:
        for p in procs:
            p.join()
        bad = [p.exitcode for p in procs if p.exitcode != 0]
        if bad:
            raise RuntimeError(f"spawned workers failed with exit codes {bad}")
    return procs
