"""DataLoader (reference: python/paddle/io/reader.py:216 DataLoader,
dataloader/dataloader_iter.py:151 _DataLoaderIterSingleProcess, :365 _DataLoaderIterMultiProcess,
paddle/fluid/operators/reader/buffered_reader.cc — async host→device staging).

Data path, MI355X-first:

* **Array datasets** (``TensorDataset`` or any dataset exposing ``_arrays``) skip per-sample
  Python entirely: each field of a batch is assembled by one native multi-threaded row gather
  (``csrc/runtime/gather.cpp``, GIL released) directly into a pinned host buffer.
* **Generic datasets** are fetched + collated in the calling thread (``num_workers=0``) or in
  forked worker processes (``num_workers>0``, ``prefetch_factor`` batches in flight per
  worker, results re-ordered by batch id).
* **Staging** (``use_buffer_reader=True`` on a GPU): a background thread pins each host batch
  and issues the H2D copy on a dedicated HIP copy stream; the consumer's stream waits on a
  per-batch event, so copies overlap the previous step's compute.  Hand-off between the
  staging thread and the training loop goes through the native bounded queue.
"""
import itertools
import multiprocessing
import threading

import numpy as np
import torch

from .dataset import IterableDataset
from .sampler import BatchSampler, _InfiniteIterableSampler
from .collate import default_collate_fn, default_convert_fn
from . import worker as _worker


def _np_to_torch(a):
    if a.dtype == np.object_:
        raise TypeError("object arrays cannot be converted to tensors")
    return torch.from_numpy(np.ascontiguousarray(a))


def _host_to_torch(obj, pin):
    """numpy leaves → torch CPU tensors (pinned when staging to a GPU)."""
    from ..core.tensor import Tensor
    if isinstance(obj, np.ndarray):
        t = _np_to_torch(obj)
        return t.pin_memory() if pin and not t.is_pinned() else t
    if isinstance(obj, Tensor):
        return obj._t
    if isinstance(obj, (np.number, np.bool_)):
        return torch.as_tensor(np.asarray(obj))
    if isinstance(obj, dict):
        return {k: _host_to_torch(v, pin) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [_host_to_torch(v, pin) for v in obj]
    return obj


def _to_device(obj, dev, non_blocking):
    if isinstance(obj, torch.Tensor):
        return obj.to(dev, non_blocking=non_blocking) if dev is not None else obj
    if isinstance(obj, dict):
        return {k: _to_device(v, dev, non_blocking) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_to_device(v, dev, non_blocking) for v in obj]
    return obj


def _wrap_tree(obj):
    from ..core.tensor import _wrap
    if isinstance(obj, torch.Tensor):
        return _wrap(obj)
    if isinstance(obj, dict):
        return {k: _wrap_tree(v) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_wrap_tree(v) for v in obj]
    return obj


def _record_stream(obj, stream):
    if isinstance(obj, torch.Tensor):
        if obj.is_cuda:
            obj.record_stream(stream)
    elif isinstance(obj, dict):
        for v in obj.values():
            _record_stream(v, stream)
    elif isinstance(obj, list):
        for v in obj:
            _record_stream(v, stream)


class DataLoader:
    def __init__(self, dataset, feed_list=None, places=None, return_list=True, batch_sampler=None, batch_size=1,
                 shuffle=False, drop_last=False, collate_fn=None, num_workers=0, use_buffer_reader=True,
                 prefetch_factor=2, use_shared_memory=True, timeout=0, worker_init_fn=None,
                 persistent_workers=False):
        self.dataset = dataset
        self.feed_list = feed_list
        self.return_list = return_list
        self.collate_fn = collate_fn
        self.num_workers = int(num_workers)
        self.use_buffer_reader = use_buffer_reader
        self.prefetch_factor = max(1, int(prefetch_factor))
        self.use_shared_memory = use_shared_memory
        self.timeout = timeout
        self.worker_init_fn = worker_init_fn
        self.persistent_workers = persistent_workers
        self.places = places
        self._iterable = isinstance(dataset, IterableDataset)
        if self.num_workers < 0:
            raise ValueError("num_workers should be a non-negative integer")
        if batch_sampler is not None:
            if batch_size != 1 or shuffle or drop_last:
                raise ValueError("batch_size/shuffle/drop_last should not be set when batch_sampler is given")
            self.batch_sampler = batch_sampler
            self.batch_size = getattr(batch_sampler, 'batch_size', None)
            self.drop_last = getattr(batch_sampler, 'drop_last', False)
            self.auto_collate = True
        elif batch_size is None:
            self.batch_sampler = None
            self.batch_size = None
            self.drop_last = drop_last
            self.auto_collate = False
        else:
            if not isinstance(batch_size, int) or batch_size <= 0:
                raise ValueError("batch_size should be None or a positive integer")
            self.batch_size = batch_size
            self.drop_last = drop_last
            self.auto_collate = True
            if self._iterable:
                if shuffle:
                    raise ValueError("IterableDataset does not support shuffle")
                self.batch_sampler = _InfiniteIterableSampler(dataset, batch_size)
            else:
                self.batch_sampler = BatchSampler(dataset=dataset, batch_size=batch_size, shuffle=shuffle,
                                                  drop_last=drop_last)

    def __len__(self):
        if self._iterable:
            raise ValueError("length of IterableDataset not supported")
        if self.batch_sampler is None:
            return len(self.dataset)
        return len(self.batch_sampler)

    def _device(self):
        from ..core.place import current_device
        p = self.places
        if isinstance(p, (list, tuple)):
            p = p[0] if p else None
        if p is not None:
            from ..core.place import to_device
            return to_device(p)
        return current_device()

    def __iter__(self):
        return _LoaderIter(self)

    def __call__(self):
        return self.__iter__()

    @staticmethod
    def from_generator(feed_list=None, capacity=None, use_double_buffer=True, iterable=True, return_list=False,
                       use_multiprocess=False, drop_last=True):
        return _GeneratorLoader(feed_list, capacity, return_list, drop_last)


class _LoaderIter:
    """One pass over the loader: host fetch (inline, native gather or worker processes) →
    optional background staging to the device → consumer."""

    def __init__(self, loader):
        self.L = loader
        self.dev = loader._device()
        self.on_gpu = self.dev is not None and self.dev.type == 'cuda'
        self._fast = (loader.auto_collate and loader.collate_fn is None and not loader._iterable and
                      hasattr(loader.dataset, '_arrays'))
        self._collate = loader.collate_fn or (default_collate_fn if loader.auto_collate else default_convert_fn)
        if loader.batch_sampler is not None:
            self._index_iter = iter(loader.batch_sampler)
        elif loader._iterable:
            self._index_iter = itertools.repeat(None)
        else:
            self._index_iter = iter(range(len(loader.dataset)))
        self._workers = []
        self._host = self._host_batches()
        self._stage_thread = None
        if self.on_gpu and loader.use_buffer_reader:
            from .._runtime import BlockingQueue
            self._q = BlockingQueue(2)
            self._copy_stream = torch.cuda.Stream(device=self.dev)
            self._stop = threading.Event()
            self._stage_thread = threading.Thread(target=self._stage_loop, daemon=True)
            self._stage_thread.start()

    # ---- host side
    def _fetch_fast(self, indices):
        from .._runtime import gather_rows
        out = []
        for a in self.L.dataset._arrays:
            buf = torch.empty((len(indices),) + a.shape[1:], dtype=_np_to_torch(a[:0]).dtype,
                              pin_memory=self.on_gpu)
            gather_rows(a, indices, buf.numpy())
            out.append(buf)
        return out

    def _fetch_inline(self, indices):
        ds = self.L.dataset
        if self.L._iterable:
            if not hasattr(self, '_ds_iter'):
                self._ds_iter = iter(ds)
            n = self.L.batch_size if self.L.auto_collate else 1
            samples = list(itertools.islice(self._ds_iter, n))
            if not samples or (self.L.auto_collate and self.L.drop_last and len(samples) < n):
                raise StopIteration
            return self._collate(samples) if self.L.auto_collate else self._collate(samples[0])
        if self.L.auto_collate:
            return self._collate([ds[i] for i in indices])
        return self._collate(ds[indices])

    def _host_batches(self):
        if self.L.num_workers == 0:
            for indices in self._index_iter:
                try:
                    yield self._fetch_fast(indices) if self._fast else self._fetch_inline(indices)
                except StopIteration:
                    return
            return
        yield from self._worker_batches()

    def _worker_batches(self):
        L = self.L
        ctx = multiprocessing.get_context('fork')
        out_q = ctx.Queue()
        done = ctx.Event()
        from ..framework import _host_seed
        base = _host_seed()
        nw = L.num_workers
        idx_qs = []
        for w in range(nw):
            iq = ctx.Queue()
            p = ctx.Process(target=_worker._worker_loop,
                            args=(L.dataset, L._iterable, iq, out_q, done, self._collate, L.auto_collate,
                                  L.worker_init_fn, w, nw, base + w, L.drop_last, L.batch_size), daemon=True)
            p.start()
            idx_qs.append(iq)
            self._workers.append(p)
        self._done = done
        self._idx_qs = idx_qs
        sent = 0
        live = set(range(nw))
        exhausted = False
        # round-robin dispatch; each batch id is pinned to one worker so iterable datasets
        # stay per-worker ordered
        inflight = {}
        results = {}
        nxt = 0

        def dispatch():
            nonlocal sent, exhausted
            if exhausted or not live:
                return False
            w = sorted(live)[sent % len(live)] if L._iterable else sent % nw
            try:
                indices = next(self._index_iter)
            except StopIteration:
                exhausted = True
                return False
            idx_qs[w].put((sent, indices))
            inflight[sent] = w
            sent += 1
            return True

        for _ in range(self.L.prefetch_factor * nw):
            if not dispatch():
                break
        try:
            while nxt < sent or (not exhausted and live):
                if nxt in results:
                    data = results.pop(nxt)
                    nxt += 1
                    dispatch()
                    if isinstance(data, _worker._IterableDatasetStopIteration):
                        live.discard(data.worker_id)
                        continue
                    yield data
                    continue
                if nxt >= sent:
                    if not dispatch():
                        break
                    continue
                try:
                    bid, data = out_q.get(timeout=L.timeout if L.timeout else 300)
                except Exception as e:  # queue.Empty
                    dead = [p.pid for p in self._workers if not p.is_alive()]
                    raise RuntimeError(f"DataLoader timed out waiting for workers (dead pids: {dead})") from e
                if isinstance(data, _worker._WorkerException):
                    data.reraise()
                results[bid] = data
        finally:
            self._shutdown_workers()

    def _shutdown_workers(self):
        if not self._workers:
            return
        self._done.set()
        for q in self._idx_qs:
            try:
                q.put(None)
            except Exception:
                pass
        for p in self._workers:
            p.join(timeout=5)
            if p.is_alive():
                p.terminate()
        self._workers = []

    # ---- staging
    def _stage_loop(self):
        try:
            with torch.cuda.device(self.dev), torch.cuda.stream(self._copy_stream):
                for host in self._host:
                    if self._stop.is_set():
                        break
                    t = _host_to_torch(host, pin=True)
                    d = _to_device(t, self.dev, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self._copy_stream)
                    if not self._q.put((d, ev, host)):
                        break
        except BaseException as e:  # noqa: BLE001 - surfaced in the consumer
            self._q.put(('__error__', e, None))
        finally:
            self._q.close()

    def __iter__(self):
        return self

    def __next__(self):
        if self._stage_thread is not None:
            ok, item = self._q.get()
            if not ok:
                raise StopIteration
            d, ev, _ = item
            if isinstance(d, str) and d == '__error__':
                raise ev
            cur = torch.cuda.current_stream(self.dev)
            cur.wait_event(ev)
            _record_stream(d, cur)
            out = d
        else:
            host = next(self._host)
            out = _to_device(_host_to_torch(host, pin=False), self.dev if self.on_gpu else None, False)
        out = _wrap_tree(out)
        if self.L.return_list or not isinstance(out, list):
            return out
        return out

    def __del__(self):
        try:
            if self._stage_thread is not None:
                self._stop.set()
                self._q.close()
            self._shutdown_workers()
        except Exception:
            pass


class _GeneratorLoader:
    """``DataLoader.from_generator`` (reference: python/paddle/io/reader.py from_generator):
    wraps a user sample/batch generator."""

    def __init__(self, feed_list, capacity, return_list, drop_last):
        self.feed_list = feed_list
        self.return_list = return_list
        self.drop_last = drop_last
        self._gen = None
        self._batch_size = None

    def set_sample_generator(self, reader, batch_size, drop_last=True, places=None):
        self._batch_size = batch_size
        self.drop_last = drop_last

        def batched():
            buf = []
            for s in reader():
                buf.append(s)
                if len(buf) == batch_size:
                    yield default_collate_fn(buf)
                    buf = []
            if buf and not drop_last:
                yield default_collate_fn(buf)
        self._gen = batched
        return self

    def set_sample_list_generator(self, reader, places=None):
        self._gen = lambda: (default_collate_fn(b) for b in reader())
        return self

    def set_batch_generator(self, reader, places=None):
        self._gen = reader
        return self

    def __iter__(self):
        from ..core.place import current_device
        dev = current_device()
        for b in self._gen():
            yield _wrap_tree(_to_device(_host_to_torch(b, pin=False), dev, False))

    def __call__(self):
        return self.__iter__()
