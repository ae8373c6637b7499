"""Parameter-server training (reference: python/paddle/distributed/ps/the_one_ps.py, fleet PS mode —
fleet.init(is_collective=False), init_server/run_server/init_worker/stop_worker, a_sync strategy,
sparse embedding tables; paddle/fluid/distributed/ps/ brpc servers with dense/sparse tables).

Design here: servers and trainers are one paddle.distributed.rpc world (TensorPipe, C++), named
``ps{i}`` and ``trainer{j}``.  Dense parameters are flattened and cut into contiguous slices, one
per server; sparse tables (embeddings) are sharded by ``row_id % num_servers`` and grow lazily.
Each table owns its optimizer state on the server (SGD / Adam / Adagrad, the reference's
``sgd``/``adam``/``adagrad`` accessors).  ``a_sync=False`` (sync): a server applies the mean of
all trainers' gradients once every trainer has pushed for that step (the handler waits on a
condition; RPC worker threads make that safe); ``a_sync=True``: every push is applied at once.

Roles come from the reference's environment contract: TRAINING_ROLE (PSERVER | TRAINER),
PADDLE_PSERVERS_IP_PORT_LIST, PADDLE_TRAINERS_NUM, PADDLE_TRAINER_ID, PADDLE_PSERVER_ID (or
POD_IP:PADDLE_PORT matched against the server list); the RPC rendezvous is
PADDLE_PS_MASTER_ENDPOINT (default: first server host, port + 1000).
"""
import os
import threading

import torch

from ...core.tensor import Tensor, _wrap, _unwrap
from ...nn.layer.layers import Layer

# ------------------------------------------------------------------ role
class PSRole:
    def __init__(self):
        e = os.environ
        self.servers = [s for s in e.get('PADDLE_PSERVERS_IP_PORT_LIST', '').split(',') if s]
        self.num_servers = len(self.servers)
        self.num_trainers = int(e.get('PADDLE_TRAINERS_NUM', '1'))
        role = e.get('TRAINING_ROLE', 'TRAINER').upper()
        self.is_server = role == 'PSERVER'
        if self.is_server:
            if 'PADDLE_PSERVER_ID' in e:
                self.index = int(e['PADDLE_PSERVER_ID'])
            else:
                me = f"{e.get('POD_IP', '127.0.0.1')}:{e.get('PADDLE_PORT', '')}"
                self.index = self.servers.index(me)
        else:
            self.index = int(e.get('PADDLE_TRAINER_ID', '0'))
        self.name = f"ps{self.index}" if self.is_server else f"trainer{self.index}"
        self.rank = self.index if self.is_server else self.num_servers + self.index
        self.world = self.num_servers + self.num_trainers
        host, port = (self.servers[0].split(':') if self.servers else ('127.0.0.1', '6170'))
        self.master = e.get('PADDLE_PS_MASTER_ENDPOINT', f"{host}:{int(port) + 1000}")


# ------------------------------------------------------------------ server-side tables
class _Opt:
    """Per-table optimizer rule applied on the server (fp32)."""

    def __init__(self, cfg):
        self.kind = cfg.get('name', 'sgd')
        self.lr = float(cfg.get('learning_rate', 0.01))
        self.b1, self.b2 = float(cfg.get('beta1', 0.9)), float(cfg.get('beta2', 0.999))
        self.eps = float(cfg.get('epsilon', 1e-8))
        self.initial_g2sum = float(cfg.get('initial_g2sum', 0.0))

    def state(self, n):
        if self.kind == 'adam':
            return {'m': torch.zeros(n), 'v': torch.zeros(n), 't': 0}
        if self.kind == 'adagrad':
            return {'g2': torch.full((n,), self.initial_g2sum)}
        return {}

    def apply(self, w, g, st):
        if self.kind == 'adam':
            st['t'] += 1
            st['m'].mul_(self.b1).add_(g, alpha=1 - self.b1)
            st['v'].mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            mh = st['m'] / (1 - self.b1 ** st['t'])
            vh = st['v'] / (1 - self.b2 ** st['t'])
            w.sub_(self.lr * mh / (vh.sqrt() + self.eps))
        elif self.kind == 'adagrad':
            st['g2'].add_(g * g)
            w.sub_(self.lr * g / (st['g2'].sqrt() + self.eps))
        else:
            w.sub_(self.lr * g)


class _DenseTable:
    def __init__(self, values, opt_cfg, sync, trainers):
        self.w = values.clone().float()
        self.opt = _Opt(opt_cfg)
        self.st = self.opt.state(self.w.numel())
        self.sync, self.trainers = sync, trainers
        self.acc, self.count, self.version = torch.zeros_like(self.w), 0, 0
        self.cv = threading.Condition()

    def push(self, g):
        g = g.float()
        with self.cv:
            if not self.sync:
                self.opt.apply(self.w, g, self.st)
                self.version += 1
                return self.version
            my_version = self.version
            self.acc.add_(g)
            self.count += 1
            if self.count == self.trainers:
                self.opt.apply(self.w, self.acc / self.trainers, self.st)
                self.acc.zero_()
                self.count = 0
                self.version += 1
                self.cv.notify_all()
            else:
                self.cv.wait_for(lambda: self.version > my_version, timeout=600)
            return self.version

    def pull(self):
        with self.cv:
            return self.w.clone()


class _SparseTable:
    def __init__(self, dim, opt_cfg, sync, trainers, init_range, seed):
        self.dim, self.opt = dim, _Opt(opt_cfg)
        self.rows, self.states = {}, {}
        self.sync, self.trainers = sync, trainers
        self.gen = torch.Generator().manual_seed(seed)
        self.init_range = init_range
        self.pending, self.count, self.version = {}, 0, 0
        self.cv = threading.Condition()

    def _row(self, i):
        r = self.rows.get(i)
        if r is None:
            r = (torch.rand(self.dim, generator=self.gen) * 2 - 1) * self.init_range
            self.rows[i] = r
            self.states[i] = self.opt.state(self.dim)
        return r

    def pull(self, ids):
        with self.cv:
            return torch.stack([self._row(int(i)) for i in ids.tolist()]) if len(ids) else torch.zeros(0, self.dim)

    def _apply(self, grads):
        for i, g in grads.items():
            self.opt.apply(self._row(i), g, self.states[i])

    def push(self, ids, g):
        with self.cv:
            merged = {}
            for i, row in zip(ids.tolist(), g.float()):
                merged[i] = merged[i] + row if i in merged else row.clone()
            if not self.sync:
                self._apply(merged)
                return
            my_version = self.version
            for i, row in merged.items():
                self.pending[i] = self.pending[i] + row if i in self.pending else row
            self.count += 1
            if self.count == self.trainers:
                self._apply({i: row / self.trainers for i, row in self.pending.items()})
                self.pending, self.count = {}, 0
                self.version += 1
                self.cv.notify_all()
            else:
                self.cv.wait_for(lambda: self.version > my_version, timeout=600)


class _Server:
    def __init__(self, role):
        self.role = role
        self.tables = {}
        self.lock = threading.Lock()
        self.stopped = threading.Event()
        self.stop_count = 0


_SERVER = [None]


def _srv():
    s = _SERVER[0]
    if s is None:
        raise RuntimeError("this process is not an initialised parameter server")
    return s


# RPC entry points (run on the server process)
def _rpc_create_dense(name, values, opt_cfg, sync, trainers):
    s = _srv()
    with s.lock:
        if name not in s.tables:  # first trainer's initial values win (all trainers share the seed)
            s.tables[name] = _DenseTable(values, opt_cfg, sync, trainers)
    return True


def _rpc_create_sparse(name, dim, opt_cfg, sync, trainers, init_range, seed):
    s = _srv()
    with s.lock:
        if name not in s.tables:
            s.tables[name] = _SparseTable(dim, opt_cfg, sync, trainers, init_range, seed + s.role.index)
    return True


def _rpc_push_dense(name, g):
    return _srv().tables[name].push(g)


def _rpc_pull_dense(name):
    return _srv().tables[name].pull()


def _rpc_pull_sparse(name, ids):
    return _srv().tables[name].pull(ids)


def _rpc_push_sparse(name, ids, g):
    _srv().tables[name].push(ids, g)
    return True


def _rpc_table_size(name):
    t = _srv().tables[name]
    return len(t.rows) if isinstance(t, _SparseTable) else t.w.numel()


def _rpc_stop():
    s = _srv()
    with s.lock:
        s.stop_count += 1
        if s.stop_count >= s.role.num_trainers:
            s.stopped.set()
    return True


# ------------------------------------------------------------------ runtime (both roles)
class PSRuntime:
    def __init__(self, role=None):
        self.role = role or PSRole()
        self._rpc_up = False

    def _start_rpc(self):
        if self._rpc_up:
            return
        from .. import rpc
        os.environ.setdefault('PADDLE_WORKER_ENDPOINT', '127.0.0.1:0')
        rpc.init_rpc(self.role.name, rank=self.role.rank, world_size=self.role.world,
                     master_endpoint=self.role.master)
        self._rpc_up = True

    # server
    def init_server(self):
        _SERVER[0] = _Server(self.role)
        self._start_rpc()

    def run_server(self):
        """Serve until every trainer called stop_worker, then leave the RPC world."""
        _srv().stopped.wait()
        from .. import rpc
        rpc.shutdown()
        self._rpc_up = False

    # trainer
    def init_worker(self):
        self._start_rpc()

    def stop_worker(self):
        from .. import rpc
        for i in range(self.role.num_servers):
            rpc.rpc_sync(f"ps{i}", _rpc_stop)
        rpc.shutdown()
        self._rpc_up = False


# ------------------------------------------------------------------ trainer-side client
class _Client:
    def __init__(self, runtime, sync=True, opt_cfg=None):
        self.rt = runtime
        self.sync = sync
        self.opt_cfg = opt_cfg or {'name': 'sgd', 'learning_rate': 0.01}
        self.dense = []  # (name, params, slices)
        self.sparse = []

    @property
    def S(self):
        return self.rt.role.num_servers

    def _cuts(self, n):
        step = (n + self.S - 1) // self.S
        return [(min(i * step, n), min((i + 1) * step, n)) for i in range(self.S)]

    def register_dense(self, name, params):
        from .. import rpc
        flat = torch.cat([_unwrap(p).detach().reshape(-1).float().cpu() for p in params])
        cuts = self._cuts(flat.numel())
        for i, (a, b) in enumerate(cuts):
            rpc.rpc_sync(f"ps{i}", _rpc_create_dense,
                         args=(name, flat[a:b].clone(), self.opt_cfg, self.sync, self.rt.role.num_trainers))
        self.dense.append((name, list(params), cuts))
        self.pull_dense()

    def pull_dense(self):
        from .. import rpc
        for name, params, cuts in self.dense:
            futs = [rpc.rpc_async(f"ps{i}", _rpc_pull_dense, args=(name,)) for i in range(len(cuts))]
            flat = torch.cat([f.wait() for f in futs])
            off = 0
            with torch.no_grad():
                for p in params:
                    t = _unwrap(p)
                    n = t.numel()
                    t.copy_(flat[off:off + n].view(t.shape).to(t.dtype))
                    off += n

    def push_dense(self):
        from .. import rpc
        for name, params, cuts in self.dense:
            g = torch.cat([(_unwrap(p).grad if _unwrap(p).grad is not None else torch.zeros_like(_unwrap(p)))
                           .detach().reshape(-1).float().cpu() for p in params])
            futs = [rpc.rpc_async(f"ps{i}", _rpc_push_dense, args=(name, g[a:b].clone()))
                    for i, (a, b) in enumerate(cuts)]
            for f in futs:
                f.wait()

    def pull_sparse(self, name, ids):
        from .. import rpc
        ids = ids.reshape(-1).cpu().long()
        out = torch.empty(ids.numel(), 0)
        owner = ids % self.S
        futs, sel = [], []
        for i in range(self.S):
            m = (owner == i).nonzero(as_tuple=True)[0]
            sel.append(m)
            futs.append(rpc.rpc_async(f"ps{i}", _rpc_pull_sparse, args=(name, ids[m])) if m.numel() else None)
        rows = None
        for i, f in enumerate(futs):
            if f is None:
                continue
            r = f.wait()
            if rows is None:
                rows = torch.empty(ids.numel(), r.shape[1])
            rows[sel[i]] = r
        return rows if rows is not None else out

    def push_sparse(self, name, ids, grads):
        from .. import rpc
        ids = ids.reshape(-1).cpu().long()
        grads = grads.reshape(ids.numel(), -1).detach().float().cpu()
        owner = ids % self.S
        futs = []
        for i in range(self.S):
            m = (owner == i).nonzero(as_tuple=True)[0]
            # sync tables expect one push per trainer per step, even an empty one
            futs.append(rpc.rpc_async(f"ps{i}", _rpc_push_sparse, args=(name, ids[m], grads[m])))
        for f in futs:
            f.wait()


_ACTIVE = {'client': None, 'embeddings': []}


class _EmbeddingPull(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, rows, layer, ids):
        ctx.layer, ctx.ids = layer, ids
        return rows.clone()

    @staticmethod
    def backward(ctx, g):
        ctx.layer._pending.append((ctx.ids, g.detach()))
        return torch.zeros_like(ctx.layer._anchor), None, None, None


class DistributedEmbedding(Layer):
    """Sparse embedding table living on the parameter servers (reference: the_one_ps sparse table
    + paddle.static.nn.sparse_embedding).  forward pulls the rows of the batch's ids; backward
    records the row gradients; the PS optimizer pushes them at step()."""

    def __init__(self, num_embeddings, embedding_dim, table_name='emb', init_range=0.01, seed=0):
        super().__init__()
        self._dim, self._name, self._range, self._seed = embedding_dim, table_name, init_range, seed
        self._client = None
        self._pending = []
        self._anchor = torch.zeros(1, requires_grad=True)

    def _bind(self, client):
        from .. import rpc
        self._client = client
        for i in range(client.S):
            rpc.rpc_sync(f"ps{i}", _rpc_create_sparse, args=(self._name, self._dim, client.opt_cfg, client.sync,
                                                              client.rt.role.num_trainers, self._range, self._seed))

    def forward(self, ids):
        if self._client is None:
            if _ACTIVE['client'] is None:
                raise RuntimeError("DistributedEmbedding needs fleet.distributed_optimizer (PS mode) first")
            self._bind(_ACTIVE['client'])
            _ACTIVE['embeddings'].append(self)
        t = _unwrap(ids)
        rows = self._client.pull_sparse(self._name, t).to(self._anchor.device)
        out = _EmbeddingPull.apply(self._anchor, rows, self, t.reshape(-1).cpu().long())
        return _wrap(out.reshape(*t.shape, self._dim))

    def push(self):
        ids = torch.cat([i for i, _ in self._pending]) if self._pending else torch.zeros(0, dtype=torch.long)
        g = torch.cat([x.reshape(-1, self._dim) for _, x in self._pending]) if self._pending else torch.zeros(0, self._dim)
        self._client.push_sparse(self._name, ids, g)
        self._pending = []


class PSOptimizer:
    """fleet.distributed_optimizer result in PS mode: step() pushes dense + sparse gradients and
    pulls the updated dense parameters (sync: after the server-side mean update)."""

    def __init__(self, optimizer, runtime, strategy=None):
        self._inner = optimizer
        sync = not bool(getattr(strategy, 'a_sync', False)) if strategy is not None else True
        name = type(optimizer).__name__.lower()
        cfg = {'name': 'adam' if name in ('adam', 'adamw') else ('adagrad' if name == 'adagrad' else 'sgd'),
               'learning_rate': float(optimizer.get_lr())}
        for k in ('_beta1', '_beta2', '_epsilon'):
            if hasattr(optimizer, k):
                cfg[k[1:]] = float(getattr(optimizer, k))
        self._client = _Client(runtime, sync=sync, opt_cfg=cfg)
        _ACTIVE['client'], _ACTIVE['embeddings'] = self._client, []
        dense = []
        for p in optimizer._parameter_list:
            dense.append(p)
        self._dense = dense
        self._registered = False

    def _register(self, model=None):
        if self._registered:
            return
        if self._dense:
            self._client.register_dense('dense', self._dense)
        self._registered = True

    def step(self):
        self._register()
        self._client.push_dense()
        for e in _ACTIVE['embeddings']:
            e.push()
        self._client.pull_dense()

    def minimize(self, loss, *a, **k):
        loss.backward()
        self.step()

    def clear_grad(self, set_to_zero=True):
        for p in self._dense:
            if _unwrap(p).grad is not None:
                _unwrap(p).grad = None

    def __getattr__(self, name):
        return getattr(self._inner, name)


__all__ = ['PSRole', 'PSRuntime', 'PSOptimizer', 'DistributedEmbedding']
