"""Multi-process loader workers (reference: python/paddle/io/dataloader/worker.py —
get_worker_info:79, WorkerInfo:158, _worker_loop:271, ParentWatchDog:63).

Workers are forked processes running dataset code only (they never touch the GPU); each
receives ``(batch_id, indices)`` work items and returns ``(batch_id, collated numpy batch)``.
"""
import os
import queue
import traceback

import numpy as np

_worker_info = None


class WorkerInfo:
    def __init__(self, **kw):
        self.__dict__.update(kw)
        self._frozen = True

    def __setattr__(self, k, v):
        if getattr(self, '_frozen', False):
            raise RuntimeError(f"Cannot assign attributes to {self.__class__.__name__} objects")
        super().__setattr__(k, v)


def get_worker_info():
    return _worker_info


class _IterableDatasetStopIteration:
    def __init__(self, worker_id):
        self.worker_id = worker_id


class _WorkerException:
    def __init__(self, worker_id, exc):
        self.worker_id = worker_id
        self.exc_type = type(exc).__name__
        self.msg = ''.join(traceback.format_exception(type(exc), exc, exc.__traceback__))

    def reraise(self):
        raise RuntimeError(f"DataLoader worker {self.worker_id} raised {self.exc_type}:\n{self.msg}")


def _to_host(obj):
    """Tensors produced in a worker are sent as numpy (they are rebuilt in the parent)."""
    from ..core.tensor import Tensor
    if isinstance(obj, Tensor):
        return obj.numpy()
    if isinstance(obj, dict):
        return {k: _to_host(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_host(v) for v in obj)
    return obj


def _worker_loop(dataset, iterable, index_q, out_q, done_event, collate_fn, auto_collate, init_fn, worker_id,
                 num_workers, seed, drop_last, batch_size):
    global _worker_info
    try:
        import random
        random.seed(seed)
        np.random.seed(seed % (2 ** 32))
        try:
            import torch
            torch.manual_seed(seed)
            torch.set_num_threads(1)
        except Exception:
            pass
        _worker_info = WorkerInfo(id=worker_id, num_workers=num_workers, dataset=dataset, seed=seed)
        if init_fn is not None:
            init_fn(worker_id)
        it = iter(dataset) if iterable else None
        parent = os.getppid()
        while not done_event.is_set():
            try:
                item = index_q.get(timeout=1.0)
            except queue.Empty:
                if os.getppid() != parent:  # parent died: exit instead of lingering
                    return
                continue
            if item is None:
                return
            bid, indices = item
            try:
                if iterable:
                    samples = []
                    for _ in range(batch_size if auto_collate else 1):
                        try:
                            samples.append(next(it))
                        except StopIteration:
                            break
                    if not samples or (auto_collate and drop_last and len(samples) < batch_size):
                        out_q.put((bid, _IterableDatasetStopIteration(worker_id)))
                        continue
                    data = collate_fn(samples) if auto_collate else collate_fn(samples[0])
                else:
                    if auto_collate:
                        data = collate_fn([dataset[i] for i in indices])
                    else:
                        data = collate_fn(dataset[indices])
                out_q.put((bid, _to_host(data)))
            except Exception as e:  # noqa: BLE001
                out_q.put((bid, _WorkerException(worker_id, e)))
    except KeyboardInterrupt:
        pass
