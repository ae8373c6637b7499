"""paddle.distributed.rpc — remote procedure calls between named workers.

Reference: python/paddle/distributed/rpc/rpc.py (init_rpc:73, rpc_sync:143, rpc_async:183,
shutdown:276, get_worker_info:307, get_all_worker_infos:337, get_current_worker_info:364), a brpc
service in C++.  Here the transport is PyTorch's native TensorPipe agent (C++, TCP/shm, tensors
travel without pickling their storage), rendezvoused through the same TCP store contract
(``master_endpoint`` / ``PADDLE_MASTER_ENDPOINT``, ``PADDLE_TRAINER_ID``, ``PADDLE_TRAINERS_NUM``).
Functions must be importable on the callee (module-level), exactly as in the reference.
"""
import os
from dataclasses import dataclass
from datetime import timedelta

import torch.distributed.rpc as _trpc

_DEFAULT_RPC_TIMEOUT = -1  # seconds; -1 = the agent default (never time out at the call site)
_state = {'name': None, 'infos': None}


@dataclass(frozen=True)
class WorkerInfo:
    name: str
    rank: int
    ip: str = '127.0.0.1'
    port: int = 0

    def __str__(self):
        return f"{{name: {self.name}, rank: {self.rank}, ip: {self.ip}, port: {self.port}}}"

    __repr__ = __str__


class FutureWrapper:
    """Result handle of rpc_async (``.wait()`` returns the remote function's return value)."""

    def __init__(self, fut):
        self._fut = fut

    def wait(self):
        return self._fut.wait()

    def done(self):
        return self._fut.done()


def init_rpc(name, rank=None, world_size=None, master_endpoint=None):
    rank = int(os.environ["PADDLE_TRAINER_ID"]) if rank is None else rank
    world_size = int(os.environ["PADDLE_TRAINERS_NUM"]) if world_size is None else world_size
    master_endpoint = master_endpoint if master_endpoint is not None else os.environ["PADDLE_MASTER_ENDPOINT"]
    timeout = int(os.getenv("FLAGS_stop_check_timeout", "900"))
    if master_endpoint.split(":")[0] in ("127.0.0.1", "localhost"):
        os.environ.setdefault("TP_SOCKET_IFNAME", "lo")  # single node: do not resolve the hostname
    # libuv TCP transport (the shm/ibv transports probe devices this pool does not expose)
    transports = os.getenv("PADDLE_RPC_TRANSPORTS", "uv").split(",")
    opts = _trpc.TensorPipeRpcBackendOptions(init_method=f"tcp://{master_endpoint}", rpc_timeout=timeout,
                                             num_worker_threads=int(os.getenv("PADDLE_RPC_THREADS", "8")),
                                             _transports=transports)
    # our rendezvous store lives at master_endpoint: under torchrun the tcp:// handler would
    # otherwise connect to the elastic agent's store instead of hosting this one
    agent = os.environ.pop("TORCHELASTIC_USE_AGENT_STORE", None)
    try:
        _trpc.init_rpc(name, rank=rank, world_size=world_size, rpc_backend_options=opts)
    finally:
        if agent is not None:
            os.environ["TORCHELASTIC_USE_AGENT_STORE"] = agent
    _state['name'] = name
    ep = os.getenv("PADDLE_WORKER_ENDPOINT", "")
    ip, port = (ep.split(":") + ["0"])[:2] if ep else ("127.0.0.1", "0")
    _state['self'] = WorkerInfo(name, rank, ip, int(port))
    infos = [_trpc.get_worker_info(w.name) for w in _trpc._get_current_rpc_agent().get_worker_infos()]
    _state['infos'] = sorted((WorkerInfo(i.name, i.id) for i in infos), key=lambda w: w.rank)


def _to(to):
    return to.name if isinstance(to, WorkerInfo) else to


def _t(timeout):
    return _trpc.constants.UNSET_RPC_TIMEOUT if timeout is None or timeout < 0 else float(timeout)


def rpc_sync(to, fn, args=None, kwargs=None, timeout=_DEFAULT_RPC_TIMEOUT):
    return _trpc.rpc_sync(_to(to), fn, args=tuple(args or ()), kwargs=dict(kwargs or {}), timeout=_t(timeout))


def rpc_async(to, fn, args=None, kwargs=None, timeout=_DEFAULT_RPC_TIMEOUT):
    return FutureWrapper(_trpc.rpc_async(_to(to), fn, args=tuple(args or ()), kwargs=dict(kwargs or {}),
                                         timeout=_t(timeout)))


def shutdown():
    """Blocks until every worker has called shutdown (graceful), then stops the agent."""
    _trpc.shutdown(graceful=True)
    _state.update(name=None, infos=None)


def get_worker_info(name):
    i = _trpc.get_worker_info(name)
    if _state.get('self') is not None and name == _state['self'].name:
        return _state['self']
    return WorkerInfo(i.name, i.id)


def get_all_worker_infos():
    return list(_state['infos'] or [])


def get_current_worker_info():
    return _state.get('self')


__all__ = ['init_rpc', 'shutdown', 'rpc_sync', 'rpc_async', 'get_worker_info', 'get_all_worker_infos',
           'get_current_worker_info', 'WorkerInfo']
