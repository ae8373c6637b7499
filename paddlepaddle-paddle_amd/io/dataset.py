"""Datasets (reference: python/paddle/io/dataloader/dataset.py — Dataset:25, IterableDataset:83,
TensorDataset:266, ComposeDataset:326, ChainDataset:392, Subset:445, random_split:485,
ConcatDataset:598)."""
import bisect
import math
import warnings

import numpy as np


class Dataset:
    def __getitem__(self, idx):
        raise NotImplementedError(f"'{self.__class__.__name__}' does not implement __getitem__")

    def __len__(self):
        raise NotImplementedError(f"'{self.__class__.__name__}' does not implement __len__")

    def __add__(self, other):
        return ConcatDataset([self, other])


class IterableDataset(Dataset):
    def __iter__(self):
        raise NotImplementedError(f"'{self.__class__.__name__}' does not implement __iter__")

    def __getitem__(self, idx):
        raise RuntimeError("'IterableDataset' does not support indexing")

    def __len__(self):
        raise TypeError("'IterableDataset' has no length")


def _np(t):
    from ..core.tensor import Tensor
    if isinstance(t, Tensor):
        return t._t.detach().cpu().numpy() if t._t.dtype.is_floating_point or t._t.dtype != _bf16() else \
            t._t.detach().float().cpu().numpy()
    return np.asarray(t)


def _bf16():
    import torch
    return torch.bfloat16


class TensorDataset(Dataset):
    """Rows of equally-long tensors.  Fields are kept as host numpy arrays so the loader can
    assemble a batch with one native multi-threaded row gather per field."""

    def __init__(self, tensors):
        from ..core.tensor import Tensor
        if not all(isinstance(t, (Tensor, np.ndarray)) for t in tensors):
            raise TypeError("TensorDataset takes paddle.Tensor or numpy.ndarray fields")
        n = tensors[0].shape[0]
        if any(t.shape[0] != n for t in tensors):
            raise ValueError("all tensors must have the same first dimension")
        self.tensors = list(tensors)
        self._arrays = [np.ascontiguousarray(_np(t)) for t in tensors]

    def __getitem__(self, index):
        return tuple(a[index] for a in self._arrays)

    def __len__(self):
        return self._arrays[0].shape[0]


def to_list(value):
    if value is None:
        return value
    if isinstance(value, (list, tuple)):
        return list(value)
    return [value]


class ComposeDataset(Dataset):
    """Zips map-style datasets: sample i is the concatenation of every dataset's fields."""

    def __init__(self, datasets):
        self.datasets = list(datasets)
        if not self.datasets:
            raise ValueError("input datasets should not be empty")
        for d in self.datasets:
            if isinstance(d, IterableDataset):
                raise TypeError("ComposeDataset only supports map-style datasets")
        if len({len(d) for d in self.datasets}) != 1:
            raise ValueError("lengths of datasets should be same")

    def __len__(self):
        return len(self.datasets[0])

    def __getitem__(self, idx):
        out = []
        for d in self.datasets:
            out.extend(to_list(d[idx]))
        return tuple(out)


class ChainDataset(IterableDataset):
    def __init__(self, datasets):
        self.datasets = list(datasets)
        for d in self.datasets:
            if not isinstance(d, IterableDataset):
                raise TypeError("ChainDataset only supports IterableDataset")

    def __iter__(self):
        for d in self.datasets:
            yield from d


class Subset(Dataset):
    def __init__(self, dataset, indices):
        self.dataset = dataset
        self.indices = list(indices)

    def __getitem__(self, idx):
        return self.dataset[self.indices[idx]]

    def __len__(self):
        return len(self.indices)


def _accumulate(xs):
    total = 0
    for x in xs:
        total += x
        yield total


def random_split(dataset, lengths, generator=None):
    lengths = list(lengths)
    if math.isclose(sum(lengths), 1) and sum(lengths) <= 1:
        sizes = []
        for i, frac in enumerate(lengths):
            if frac < 0 or frac > 1:
                raise ValueError(f"Fraction at index {i} is not between 0 and 1")
            sizes.append(int(math.floor(len(dataset) * frac)))
        for i in range(len(dataset) - sum(sizes)):
            sizes[i % len(sizes)] += 1
        for i, n in enumerate(sizes):
            if n == 0:
                warnings.warn(f"Length of split at index {i} is 0. This might result in an empty dataset.")
        lengths = sizes
    if sum(lengths) != len(dataset):
        raise ValueError("Sum of input lengths does not equal the length of the input dataset!")
    from ..tensor.logic import randperm
    perm = randperm(sum(lengths)).numpy().tolist()
    return [Subset(dataset, perm[end - n:end]) for end, n in zip(_accumulate(lengths), lengths)]


class ConcatDataset(Dataset):
    def __init__(self, datasets):
        self.datasets = list(datasets)
        if not self.datasets:
            raise ValueError("datasets should not be an empty iterable")
        for d in self.datasets:
            if isinstance(d, IterableDataset):
                raise TypeError("ConcatDataset does not support IterableDataset")
        self.cumulative_sizes = list(_accumulate(len(d) for d in self.datasets))

    def __len__(self):
        return self.cumulative_sizes[-1]

    def __getitem__(self, idx):
        if idx < 0:
            if -idx > len(self):
                raise ValueError("absolute value of index should not exceed dataset length")
            idx = len(self) + idx
        k = bisect.bisect_right(self.cumulative_sizes, idx)
        base = 0 if k == 0 else self.cumulative_sizes[k - 1]
        return self.datasets[k][idx - base]
