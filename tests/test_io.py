"""paddle.io: datasets, samplers, DataLoader (inline, native fast path, worker processes)."""
import numpy as np
import pytest

import paddle
from paddle.io import (Dataset, IterableDataset, TensorDataset, DataLoader, BatchSampler, DistributedBatchSampler,
                       RandomSampler, SequenceSampler, Subset, random_split, ConcatDataset, ComposeDataset,
                       ChainDataset, WeightedRandomSampler, SubsetRandomSampler, get_worker_info)


class RandomDataset(Dataset):
    def __init__(self, n):
        self.n = n

    def __getitem__(self, i):
        return np.full([4], i, dtype=np.float32), np.array([i % 3], dtype=np.int64)

    def __len__(self):
        return self.n


class Stream(IterableDataset):
    def __init__(self, n):
        self.n = n

    def __iter__(self):
        info = get_worker_info()
        lo, step = (0, 1) if info is None else (info.id, info.num_workers)
        for i in range(lo, self.n, step):
            yield np.array([i], dtype=np.float32)


@pytest.mark.parametrize("workers", [0, 2])
def test_map_dataset_order_and_shapes(workers):
    dl = DataLoader(RandomDataset(10), batch_size=4, num_workers=workers)
    assert len(dl) == 3
    seen = []
    for x, y in dl:
        assert isinstance(x, paddle.Tensor) and x.shape[1:] == [4]
        seen.extend(x.numpy()[:, 0].tolist())
        assert y.dtype == paddle.int64
    assert seen == list(range(10))


def test_tensor_dataset_native_gather_matches():
    xs = np.random.rand(50, 3, 5).astype(np.float32)
    ys = np.arange(50, dtype=np.int64)
    ds = TensorDataset([paddle.to_tensor(xs), ys])
    dl = DataLoader(ds, batch_size=8, shuffle=True, drop_last=True)
    n = 0
    for x, y in dl:
        np.testing.assert_array_equal(x.numpy(), xs[y.numpy()])
        n += 1
    assert n == 6


@pytest.mark.parametrize("workers", [0, 2])
def test_iterable_dataset(workers):
    dl = DataLoader(Stream(10), batch_size=3, num_workers=workers)
    got = sorted(v for b in dl for v in b.numpy().reshape(-1).tolist())
    assert got == list(range(10))


def test_batch_sampler_and_distributed():
    ds = RandomDataset(11)
    bs = BatchSampler(ds, batch_size=4, drop_last=False)
    assert [len(b) for b in bs] == [4, 4, 3]
    r0 = list(DistributedBatchSampler(ds, 2, num_replicas=2, rank=0))
    r1 = list(DistributedBatchSampler(ds, 2, num_replicas=2, rank=1))
    a = [i for b in r0 for i in b]
    b = [i for b_ in r1 for i in b_]
    assert len(a) == len(b) == 6
    assert set(a) | set(b) == set(range(11))
    s = DistributedBatchSampler(ds, 2, num_replicas=2, rank=0, shuffle=True)
    e0 = list(s)
    e1 = list(s)
    assert e0 != e1  # epoch advances the permutation


def test_samplers_and_dataset_combinators():
    paddle.seed(3)
    ds = RandomDataset(10)
    assert sorted(RandomSampler(ds)) == list(range(10))
    assert list(SequenceSampler(ds)) == list(range(10))
    assert len(list(RandomSampler(ds, replacement=True, num_samples=25))) == 25
    w = list(WeightedRandomSampler([0.0, 0.0, 1.0], 5))
    assert w == [2] * 5
    assert sorted(SubsetRandomSampler([1, 5, 7])) == [1, 5, 7]
    a, b = random_split(ds, [0.7, 0.3])
    assert len(a) == 7 and len(b) == 3 and set(a.indices) | set(b.indices) == set(range(10))
    c = ConcatDataset([ds, Subset(ds, [0, 1])])
    assert len(c) == 12 and c[11][0][0] == 1
    comp = ComposeDataset([ds, ds])
    assert len(comp[0]) == 4
    ch = list(ChainDataset([Stream(2), Stream(3)]))
    assert len(ch) == 5


def test_dict_collate_and_batch_size_none():
    class D(Dataset):
        def __getitem__(self, i):
            return {'a': np.ones(2, np.float32) * i, 'b': i}

        def __len__(self):
            return 5
    out = list(DataLoader(D(), batch_size=5))[0]
    assert out['a'].shape == [5, 2] and out['b'].numpy().tolist() == [0, 1, 2, 3, 4]
    out = list(DataLoader(D(), batch_size=None))
    assert len(out) == 5


def test_worker_error_is_raised():
    class Bad(Dataset):
        def __getitem__(self, i):
            raise ValueError("boom")

        def __len__(self):
            return 4
    with pytest.raises(RuntimeError, match="boom"):
        list(DataLoader(Bad(), batch_size=2, num_workers=1))


def test_from_generator():
    loader = DataLoader.from_generator(capacity=4)
    loader.set_sample_generator(lambda: ((np.ones(3, np.float32) * i,) for i in range(5)), batch_size=2,
                                drop_last=True)
    assert len(list(loader())) == 2
