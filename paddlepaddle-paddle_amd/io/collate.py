"""Batch collation (reference: python/paddle/io/dataloader/collate.py:25 default_collate_fn,
:83 default_convert_fn).  Collation produces host numpy arrays; conversion to device tensors
happens once per batch in the loader's staging step."""
import numbers
from collections.abc import Mapping, Sequence

import numpy as np


def default_collate_fn(batch):
    from ..core.tensor import Tensor
    sample = batch[0]
    if isinstance(sample, np.ndarray):
        return np.stack(batch, axis=0)
    if isinstance(sample, Tensor):
        from ..tensor.manipulation import stack
        return stack(batch, axis=0)
    if isinstance(sample, (bool, np.bool_)):
        return np.array(batch)
    if isinstance(sample, (numbers.Number, np.number)):
        return np.array(batch)
    if isinstance(sample, (str, bytes)):
        return batch
    if isinstance(sample, Mapping):
        return {k: default_collate_fn([d[k] for d in batch]) for k in sample}
    if isinstance(sample, Sequence):
        n = len(sample)
        if not all(len(s) == n for s in batch):
            raise RuntimeError("fields number not same among samples in a batch")
        return [default_collate_fn(list(f)) for f in zip(*batch)]
    raise TypeError(f"batch data can only contain: tensor, numpy.ndarray, dict, list, number, but got {type(sample)}")


def default_convert_fn(batch):
    from ..core.tensor import Tensor
    if isinstance(batch, (Tensor, np.ndarray, str, bytes)):
        return batch
    if isinstance(batch, Mapping):
        return {k: default_convert_fn(v) for k, v in batch.items()}
    if isinstance(batch, Sequence):
        return [default_convert_fn(b) for b in batch]
    return batch
