"""Collective communication API (reference: python/paddle/distributed/communication/*.py).

Backed by torch.distributed process groups: backend "nccl" IS RCCL on ROCm (point-to-point
xGMI links between the 8 MI355X of a node), "gloo" for CPU tensors / CPU tests.
``sync_op=False`` returns a task with ``wait()``; otherwise the collective is enqueued on the
communicator stream and ordered against the caller's stream (RCCL semantics).
"""
import pickle

import numpy as np
import torch
import torch.distributed as dist

from ..core.tensor import Tensor, _wrap, _unwrap


class ReduceOp:
    SUM = 0
    MAX = 1
    MIN = 2
    PROD = 3
    AVG = 4


_OPS = {ReduceOp.SUM: dist.ReduceOp.SUM, ReduceOp.MAX: dist.ReduceOp.MAX, ReduceOp.MIN: dist.ReduceOp.MIN,
        ReduceOp.PROD: dist.ReduceOp.PRODUCT, ReduceOp.AVG: dist.ReduceOp.AVG}


def _op(op):
    if isinstance(op, dist.ReduceOp.RedOpType if hasattr(dist.ReduceOp, 'RedOpType') else ()):
        return op
    return _OPS.get(op, op)


class Group:
    """paddle.distributed.Group: wraps a torch ProcessGroup plus the global ranks it contains."""

    def __init__(self, rank_in_group, gid, ranks, pg=None, name=None):
        self.rank = rank_in_group
        self.id = gid
        self.ranks = list(ranks)
        self.nranks = len(ranks)
        self.world_size = self.nranks
        self.pg = pg
        self.name = name or f"group_{gid}"

    @property
    def process_group(self):
        return self.pg

    def is_member(self):
        return self.rank >= 0

    def get_group_rank(self, rank):
        return self.ranks.index(rank) if rank in self.ranks else -1

    def __repr__(self):
        return f"Group(id={self.id}, nranks={self.nranks}, rank={self.rank}, ranks={self.ranks})"


_groups = {}
_global = [None]


def _backend_for_default():
    return 'nccl' if torch.cuda.is_available() else 'gloo'


def _world():
    if _global[0] is None:
        if dist.is_available() and dist.is_initialized():
            ws = dist.get_world_size()
            _global[0] = Group(dist.get_rank(), 0, list(range(ws)), None, 'global')
            _groups[0] = _global[0]
        else:
            _global[0] = Group(0, 0, [0], None, 'global')
    return _global[0]


def _pg(group):
    if group is None:
        return None
    if isinstance(group, Group):
        return group.pg
    return group


def is_initialized():
    return dist.is_available() and dist.is_initialized()


def is_available():
    return dist.is_available()


def get_rank(group=None):
    if not is_initialized():
        return 0
    if group is not None:
        return group.rank
    return dist.get_rank()


def get_world_size(group=None):
    if not is_initialized():
        return 1
    if group is not None:
        return group.nranks
    return dist.get_world_size()


def get_backend(group=None):
    if not is_initialized():
        return 'undefined'
    b = dist.get_backend(_pg(group))
    return 'NCCL' if b == 'nccl' else b.upper()


def new_group(ranks=None, backend=None, timeout=None):
    if not is_initialized():
        g = Group(0, len(_groups) + 1, ranks or [0], None)
        _groups[g.id] = g
        return g
    ranks = sorted(ranks) if ranks is not None else list(range(dist.get_world_size()))
    kw = {}
    if timeout is not None:
        import datetime
        kw['timeout'] = timeout if isinstance(timeout, datetime.timedelta) else datetime.timedelta(seconds=timeout)
    if backend is not None:
        kw['backend'] = {'nccl': 'nccl', 'rccl': 'nccl', 'gloo': 'gloo'}.get(str(backend).lower(), backend)
    pg = dist.new_group(ranks=ranks, **kw)
    me = dist.get_rank()
    gid = max(list(_groups.keys()) + [0]) + 1
    g = Group(ranks.index(me) if me in ranks else -1, gid, ranks, pg)
    _groups[gid] = g
    return g


def get_group(id=0):  # noqa: A002
    if id == 0:
        return _world()
    return _groups.get(id)


def destroy_process_group(group=None):
    if group is None:
        if is_initialized():
            dist.destroy_process_group()
        _groups.clear()
        _global[0] = None
    else:
        if group.pg is not None:
            dist.destroy_process_group(group.pg)
        _groups.pop(group.id, None)


class _Task:
    def __init__(self, work=None, post=None):
        self._work, self._post = work, post

    def wait(self):
        if self._work is not None:
            self._work.wait()
        if self._post is not None:
            self._post()
            self._post = None
        return True

    def is_completed(self):
        return self._work is None or self._work.is_completed()


def _ret(work, sync_op, post=None):
    if sync_op:
        if work is not None:
            work.wait()
        if post is not None:
            post()
        return None
    return _Task(work, post)


def _single():
    return not is_initialized()


def all_reduce(tensor, op=ReduceOp.SUM, group=None, sync_op=True):
    if _single():
        return None if sync_op else _Task()
    t = _unwrap(tensor)
    if op == ReduceOp.AVG and dist.get_backend(_pg(group)) == 'gloo':
        w = dist.all_reduce(t, dist.ReduceOp.SUM, group=_pg(group), async_op=not sync_op)
        n = get_world_size(group)
        return _ret(w, sync_op, lambda: t.div_(n))
    w = dist.all_reduce(t, _op(op), group=_pg(group), async_op=not sync_op)
    return _ret(w, sync_op)


def all_gather(tensor_list, tensor, group=None, sync_op=True):
    t = _unwrap(tensor)
    n = get_world_size(group)
    if _single():
        tensor_list.clear() if isinstance(tensor_list, list) else None
        tensor_list.append(_wrap(t.clone()))
        return None
    if isinstance(tensor_list, Tensor):  # all_gather into one pre-allocated tensor
        w = dist.all_gather_into_tensor(_unwrap(tensor_list), t.contiguous(), group=_pg(group), async_op=not sync_op)
        return _ret(w, sync_op)
    outs = [torch.empty_like(t) for _ in range(n)]
    w = dist.all_gather(outs, t.contiguous(), group=_pg(group), async_op=not sync_op)

    def post():
        tensor_list.clear()
        tensor_list.extend(_wrap(o) for o in outs)
    return _ret(w, sync_op, post)


def all_gather_object(object_list, obj, group=None):
    if _single():
        object_list.clear()
        object_list.append(obj)
        return
    out = [None] * get_world_size(group)
    dist.all_gather_object(out, obj, group=_pg(group))
    object_list.clear()
    object_list.extend(out)


def broadcast(tensor, src, group=None, sync_op=True):
    if _single():
        return None
    w = dist.broadcast(_unwrap(tensor), src, group=_pg(group), async_op=not sync_op)
    return _ret(w, sync_op)


def broadcast_object_list(object_list, src, group=None):
    if _single():
        return
    dist.broadcast_object_list(object_list, src, group=_pg(group))


def reduce(tensor, dst, op=ReduceOp.SUM, group=None, sync_op=True):
    if _single():
        return None
    w = dist.reduce(_unwrap(tensor), dst, _op(op), group=_pg(group), async_op=not sync_op)
    return _ret(w, sync_op)


def reduce_scatter(tensor, tensor_list, op=ReduceOp.SUM, group=None, sync_op=True):
    out = _unwrap(tensor)
    if _single():
        src = _unwrap(tensor_list[0]) if isinstance(tensor_list, (list, tuple)) else _unwrap(tensor_list)
        out.copy_(src.reshape(out.shape))
        return None
    if isinstance(tensor_list, (list, tuple)):
        inp = torch.cat([_unwrap(x).reshape(-1) for x in tensor_list])
    else:
        inp = _unwrap(tensor_list).reshape(-1)
    w = dist.reduce_scatter_tensor(out.reshape(-1) if out.is_contiguous() else out, inp, _op(op), group=_pg(group),
                                   async_op=not sync_op)
    return _ret(w, sync_op)


def _reduce_scatter_base(output, input, op=ReduceOp.SUM, group=None, sync_op=True):  # noqa: A002
    return reduce_scatter(output, input, op, group, sync_op)


def scatter(tensor, tensor_list=None, src=0, group=None, sync_op=True):
    t = _unwrap(tensor)
    if _single():
        t.copy_(_unwrap(tensor_list[0]))
        return None
    me = get_rank(group) if group is not None else dist.get_rank()
    lst = [_unwrap(x) for x in tensor_list] if me == src and tensor_list is not None else None
    gsrc = group.ranks[src] if group is not None else src
    w = dist.scatter(t, lst, src=gsrc, group=_pg(group), async_op=not sync_op)
    return _ret(w, sync_op)


def scatter_object_list(out_object_list, in_object_list=None, src=0, group=None):
    if _single():
        out_object_list.clear()
        out_object_list.append(in_object_list[0])
        return
    out = [None]
    dist.scatter_object_list(out, in_object_list, src=src, group=_pg(group))
    out_object_list.clear()
    out_object_list.extend(out)


def gather(tensor, gather_list=None, dst=0, group=None, sync_op=True):
    t = _unwrap(tensor)
    if _single():
        if gather_list is not None:
            gather_list.clear()
            gather_list.append(_wrap(t.clone()))
        return None
    n = get_world_size(group)
    me = get_rank(group) if group is not None else dist.get_rank()
    outs = [torch.empty_like(t) for _ in range(n)] if me == dst else None
    if dist.get_backend(_pg(group)) == 'nccl':
        # RCCL has no native gather: all_gather then keep on dst (fine at 288 GB/GPU)
        allo = [torch.empty_like(t) for _ in range(n)]
        w = dist.all_gather(allo, t.contiguous(), group=_pg(group), async_op=not sync_op)
        outs = allo if me == dst else None
    else:
        gdst = group.ranks[dst] if group is not None else dst
        w = dist.gather(t.contiguous(), outs, dst=gdst, group=_pg(group), async_op=not sync_op)

    def post():
        if gather_list is not None and outs is not None:
            gather_list.clear()
            gather_list.extend(_wrap(o) for o in outs)
    return _ret(w, sync_op, post)


def all_to_all_tensors(outs, ins, pg=None, async_op=False):
    """torch all_to_all, with a P2P fallback for backends without it (gloo, CPU tests):
    every pair exchanges its chunk with one batched isend/irecv round."""
    if dist.get_backend(pg) != 'gloo':
        return dist.all_to_all(outs, ins, group=pg, async_op=async_op)
    me = dist.get_rank(pg)
    n = dist.get_world_size(pg)
    ranks = dist.get_process_group_ranks(pg) if pg is not None else list(range(n))
    ops = []
    for i in range(n):
        if i == me:
            outs[i].copy_(ins[i])
            continue
        ops.append(dist.P2POp(dist.isend, ins[i], ranks[i], group=pg))
        ops.append(dist.P2POp(dist.irecv, outs[i], ranks[i], group=pg))
    for w in dist.batch_isend_irecv(ops) if ops else []:
        w.wait()
    return None


def alltoall(in_tensor_list, out_tensor_list, group=None, sync_op=True):
    ins = [_unwrap(x).contiguous() for x in in_tensor_list]
    if _single():
        out_tensor_list.clear()
        out_tensor_list.extend(_wrap(x.clone()) for x in ins)
        return None
    outs = [torch.empty_like(x) for x in ins]
    w = all_to_all_tensors(outs, ins, _pg(group), async_op=not sync_op)

    def post():
        out_tensor_list.clear()
        out_tensor_list.extend(_wrap(o) for o in outs)
    return _ret(w, sync_op, post)


def alltoall_single(in_tensor, out_tensor, in_split_sizes=None, out_split_sizes=None, group=None, sync_op=True):
    if _single():
        _unwrap(out_tensor).copy_(_unwrap(in_tensor))
        return None
    w = dist.all_to_all_single(_unwrap(out_tensor), _unwrap(in_tensor), out_split_sizes, in_split_sizes,
                               group=_pg(group), async_op=not sync_op)
    return _ret(w, sync_op)


def send(tensor, dst=0, group=None, sync_op=True):
    gdst = group.ranks[dst] if group is not None else dst
    if sync_op:
        dist.send(_unwrap(tensor), gdst, group=_pg(group))
        return None
    return _Task(dist.isend(_unwrap(tensor), gdst, group=_pg(group)))


def recv(tensor, src=0, group=None, sync_op=True):
    gsrc = group.ranks[src] if group is not None else src
    if sync_op:
        dist.recv(_unwrap(tensor), gsrc, group=_pg(group))
        return None
    return _Task(dist.irecv(_unwrap(tensor), gsrc, group=_pg(group)))


def isend(tensor, dst, group=None):
    return send(tensor, dst, group, sync_op=False)


def irecv(tensor, src=None, group=None):
    return recv(tensor, src, group, sync_op=False)


class P2POp:
    def __init__(self, op, tensor, peer, group=None):
        self.op, self.tensor, self.peer, self.group = op, tensor, peer, group


def batch_isend_irecv(p2p_op_list):
    ops = []
    for p in p2p_op_list:
        fn = dist.isend if p.op in (isend, dist.isend) else dist.irecv
        peer = p.group.ranks[p.peer] if p.group is not None else p.peer
        ops.append(dist.P2POp(fn, _unwrap(p.tensor), peer, group=_pg(p.group)))
    works = dist.batch_isend_irecv(ops)
    return [_Task(w) for w in works]


def barrier(group=None):
    if _single():
        return
    if dist.get_backend(_pg(group)) == 'nccl':
        dist.barrier(group=_pg(group), device_ids=[torch.cuda.current_device()])
    else:
        dist.barrier(group=_pg(group))


def wait(tensor, group=None, use_calc_stream=True):
    if torch.cuda.is_available() and _unwrap(tensor).is_cuda:
        torch.cuda.current_stream().synchronize() if not use_calc_stream else None


def split(x, size, operation, axis=0, num_partitions=1, gather_out=True, weight_attr=None, bias_attr=None,
          name=None):
    from .fleet.layers.mpu import _split_api
    return _split_api(x, size, operation, axis, num_partitions, gather_out, weight_attr, bias_attr, name)


def convert_object_to_tensor(obj):
    data = np.frombuffer(pickle.dumps(obj), dtype=np.uint8)
    return _wrap(torch.from_numpy(data.copy())), _wrap(torch.tensor([data.size]))


# ---- collective watchdog: every public collective registers with distributed/watchdog.py
def _watched(fn):
    import functools
    from . import watchdog

    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        if not watchdog.enabled() or _single():
            return fn(*args, **kwargs)
        grp = kwargs.get('group')
        ranks = grp.ranks if isinstance(grp, Group) else list(range(get_world_size()))
        first = next((a for a in args if hasattr(a, 'shape')), None)
        tid = watchdog.begin(fn.__name__, ranks, first)
        try:
            r = fn(*args, **kwargs)
        except BaseException:
            watchdog.end(tid)
            raise
        if isinstance(r, _Task) and r._work is not None:
            watchdog.attach(tid, r._work)
        else:
            watchdog.end(tid)
        return r
    return wrapper


for _name in ('all_reduce', 'all_gather', 'all_gather_object', 'broadcast', 'broadcast_object_list', 'reduce',
              'reduce_scatter', 'scatter', 'scatter_object_list', 'gather', 'alltoall', 'alltoall_single', 'send',
              'recv', 'barrier'):
    globals()[_name] = _watched(globals()[_name])


class stream:
    """paddle.distributed.stream.* variants (use_calc_stream runs on the caller's stream)."""
    all_reduce = staticmethod(lambda tensor, op=ReduceOp.SUM, group=None, sync_op=True, use_calc_stream=False:
                              all_reduce(tensor, op, group, sync_op))
    all_gather = staticmethod(lambda tensor_or_tensor_list, tensor, group=None, sync_op=True, use_calc_stream=False:
                              all_gather(tensor_or_tensor_list, tensor, group, sync_op))
    reduce_scatter = staticmethod(lambda tensor, tensor_or_tensor_list, op=ReduceOp.SUM, group=None, sync_op=True,
                                  use_calc_stream=False: reduce_scatter(tensor, tensor_or_tensor_list, op, group,
                                                                        sync_op))
    broadcast = staticmethod(lambda tensor, src, group=None, sync_op=True, use_calc_stream=False:
                             broadcast(tensor, src, group, sync_op))
    reduce = staticmethod(lambda tensor, dst=0, op=ReduceOp.SUM, group=None, sync_op=True, use_calc_stream=False:
                          reduce(tensor, dst, op, group, sync_op))
    alltoall = staticmethod(lambda out_tensor_or_tensor_list, in_tensor_or_tensor_list, group=None, sync_op=True,
                            use_calc_stream=False: alltoall(in_tensor_or_tensor_list, out_tensor_or_tensor_list,
                                                            group, sync_op))
    alltoall_single = staticmethod(lambda out_tensor, in_tensor, out_split_sizes=None, in_split_sizes=None,
                                   group=None, sync_op=True, use_calc_stream=False:
                                   alltoall_single(in_tensor, out_tensor, in_split_sizes, out_split_sizes, group,
                                                   sync_op))
    send = staticmethod(lambda tensor, dst=0, group=None, sync_op=True, use_calc_stream=False:
                        send(tensor, dst, group, sync_op))
    recv = staticmethod(lambda tensor, src=0, group=None, sync_op=True, use_calc_stream=False:
                        recv(tensor, src, group, sync_op))
    scatter = staticmethod(lambda tensor, tensor_or_tensor_list=None, src=0, group=None, sync_op=True,
                           use_calc_stream=False: scatter(tensor, tensor_or_tensor_list, src, group, sync_op))
    gather = staticmethod(lambda tensor, gather_list=None, dst=0, group=None, sync_op=True, use_calc_stream=False:
                          gather(tensor, gather_list, dst, group, sync_op))


def _register_stream_module():
    """``paddle.distributed.communication.stream`` as an importable module (reference:
    python/paddle/distributed/communication/stream/__init__.py)."""
    import sys
    import types
    mod = types.ModuleType(__name__ + '.stream', stream.__doc__)
    for k, v in vars(stream).items():
        if not k.startswith('_'):
            setattr(mod, k, v.__func__ if isinstance(v, staticmethod) else v)
    mod.__all__ = [k for k in vars(mod) if not k.startswith('_')]
    sys.modules[mod.__name__] = mod
    return mod


_register_stream_module()
