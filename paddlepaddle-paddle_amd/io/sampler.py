"""Samplers (reference: python/paddle/io/dataloader/sampler.py — Sampler:21, SequenceSampler:97,
RandomSampler:151, WeightedRandomSampler:289, SubsetRandomSampler:346; batch_sampler.py —
BatchSampler:23, DistributedBatchSampler:170)."""
import math

import numpy as np


class Sampler:
    def __init__(self, data_source=None):
        self.data_source = data_source

    def __iter__(self):
        raise NotImplementedError

    def __len__(self):
        raise NotImplementedError


class SequenceSampler(Sampler):
    def __iter__(self):
        return iter(range(len(self.data_source)))

    def __len__(self):
        return len(self.data_source)


def _np_gen(generator):
    if generator is None:
        from ..framework import _host_seed
        return np.random.default_rng(_host_seed())
    if isinstance(generator, (int, np.integer)):
        return np.random.default_rng(int(generator))
    return generator


class RandomSampler(Sampler):
    def __init__(self, data_source, replacement=False, num_samples=None, generator=None):
        super().__init__(data_source)
        self.replacement = replacement
        self._num_samples = num_samples
        self.generator = generator
        if not isinstance(replacement, bool):
            raise TypeError("replacement should be a boolean value")
        if num_samples is not None and not replacement:
            raise ValueError("num_samples should not be specified while replacement is False")
        if self.num_samples <= 0:
            raise ValueError(f"num_samples should be a positive integer, but got {self.num_samples}")

    @property
    def num_samples(self):
        return len(self.data_source) if self._num_samples is None else self._num_samples

    def __iter__(self):
        n = len(self.data_source)
        if self.generator is not None and hasattr(self.generator, '__next__'):
            for _ in range(self.num_samples):
                yield int(next(self.generator))
            return
        g = _np_gen(self.generator)
        if self.replacement:
            yield from g.integers(0, n, self.num_samples).tolist()
        else:
            yield from g.permutation(n).tolist()

    def __len__(self):
        return self.num_samples


class WeightedRandomSampler(Sampler):
    def __init__(self, weights, num_samples, replacement=True):
        if not isinstance(num_samples, int) or num_samples <= 0:
            raise ValueError("num_samples should be a positive integer")
        from ..core.tensor import Tensor
        w = weights.numpy() if isinstance(weights, Tensor) else np.asarray(weights)
        self.weights = w.astype(np.float64).reshape(-1)
        if (self.weights < 0).any():
            raise ValueError("weights should be non-negative")
        if not replacement and num_samples > len(self.weights):
            raise ValueError("num_samples should not exceed the number of weights without replacement")
        self.num_samples = num_samples
        self.replacement = replacement

    def __iter__(self):
        p = self.weights / self.weights.sum()
        g = _np_gen(None)
        return iter(g.choice(len(p), self.num_samples, replace=self.replacement, p=p).tolist())

    def __len__(self):
        return self.num_samples


class SubsetRandomSampler(Sampler):
    def __init__(self, indices, generator=None):
        if len(indices) == 0:
            raise ValueError("The length of `indices` in SubsetRandomSampler should be greater than 0.")
        self.indices = list(indices)
        self.generator = generator

    def __iter__(self):
        g = _np_gen(self.generator)
        for i in g.permutation(len(self.indices)).tolist():
            yield self.indices[i]

    def __len__(self):
        return len(self.indices)


class BatchSampler(Sampler):
    def __init__(self, dataset=None, sampler=None, shuffle=False, batch_size=1, drop_last=False):
        if dataset is None:
            if sampler is None:
                raise ValueError("either dataset or sampler should be set")
            if shuffle:
                raise ValueError("shuffle should be False when sampler is set")
            self.sampler = sampler
        else:
            if sampler is not None:
                raise ValueError("should not set both dataset and sampler")
            from .dataset import IterableDataset
            if isinstance(dataset, IterableDataset):
                raise TypeError("dataset should not be an IterableDataset")
            self.sampler = RandomSampler(dataset) if shuffle else SequenceSampler(dataset)
        if not isinstance(batch_size, int) or batch_size <= 0:
            raise ValueError("batch_size should be a positive integer")
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.drop_last = drop_last

    def __iter__(self):
        batch = []
        for idx in self.sampler:
            batch.append(idx)
            if len(batch) == self.batch_size:
                yield batch
                batch = []
        if batch and not self.drop_last:
            yield batch

    def __len__(self):
        n = len(self.sampler)
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size


class _InfiniteIterableSampler:
    def __init__(self, dataset, batch_size=1):
        self.dataset = dataset
        self.batch_size = batch_size

    def __iter__(self):
        while True:
            yield [None] * self.batch_size


class DistributedBatchSampler(BatchSampler):
    """Each rank takes a disjoint, equally long slice (padded by wrap-around) of the index
    list; with ``shuffle`` the permutation is seeded by the epoch so all ranks agree."""

    def __init__(self, dataset, batch_size, num_replicas=None, rank=None, shuffle=False, drop_last=False):
        self.dataset = dataset
        if not isinstance(batch_size, int) or batch_size <= 0:
            raise ValueError("batch_size should be a positive integer")
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.drop_last = drop_last
        from ..distributed.parallel import ParallelEnv
        env = ParallelEnv()
        self.nranks = num_replicas if num_replicas is not None else env.nranks
        self.local_rank = rank if rank is not None else env.local_rank
        self.epoch = 0
        self.num_samples = int(math.ceil(len(self.dataset) / self.nranks))
        self.total_size = self.num_samples * self.nranks

    def __iter__(self):
        n = len(self.dataset)
        idx = list(range(n))
        pad = self.total_size - n
        idx += (idx * math.ceil(pad / max(n, 1)))[:pad]
        if self.shuffle:
            np.random.RandomState(self.epoch).shuffle(idx)
            self.epoch += 1
        if self.nranks > 1:
            # whole batches round-robin over ranks, then the tail split evenly
            stride = self.batch_size * self.nranks
            tail = self.total_size % stride
            local = []
            for i in range(self.local_rank * self.batch_size, len(idx) - tail, stride):
                local.extend(idx[i:i + self.batch_size])
            rest = idx[len(idx) - tail:]
            per = tail // self.nranks
            local.extend(rest[self.local_rank * per:(self.local_rank + 1) * per])
            idx = local
        batch = []
        for i in idx:
            batch.append(i)
            if len(batch) == self.batch_size:
                yield batch
                batch = []
        if batch and not self.drop_last:
            yield batch

    def __len__(self):
        n = self.num_samples + (0 if self.drop_last else self.batch_size - 1)
        return n // self.batch_size

    def set_epoch(self, epoch):
        self.epoch = epoch
