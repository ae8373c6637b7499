"""paddle.io (reference: python/paddle/io/__init__.py)."""
from .dataset import (Dataset, IterableDataset, TensorDataset, ComposeDataset, ChainDataset,  # noqa: F401
                      Subset, random_split, ConcatDataset)
from .sampler import (Sampler, SequenceSampler, RandomSampler, WeightedRandomSampler,  # noqa: F401
                      SubsetRandomSampler, BatchSampler, DistributedBatchSampler)
from .collate import default_collate_fn, default_convert_fn  # noqa: F401
from .worker import get_worker_info, WorkerInfo  # noqa: F401
from .dataloader import DataLoader  # noqa: F401

__all__ = ['Dataset', 'IterableDataset', 'TensorDataset', 'ComposeDataset', 'ChainDataset', 'Subset',
           'random_split', 'ConcatDataset', 'Sampler', 'SequenceSampler', 'RandomSampler',
           'WeightedRandomSampler', 'SubsetRandomSampler', 'BatchSampler', 'DistributedBatchSampler',
           'DataLoader', 'get_worker_info']
