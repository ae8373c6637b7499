"""fleet datasets (InMemoryDataset / QueueDataset over MultiSlot slot files, pipe_command through a
MultiSlotDataGenerator script) feeding Executor.train_from_dataset; sparse-table entry configs
(reference distributed/fleet/dataset/dataset.py, base/executor.py train_from_dataset,
distributed/entry_attr.py)."""
import os
import sys

import numpy as np
import pytest

import paddle


@pytest.fixture
def static_mode():
    paddle.enable_static()
    yield
    paddle.disable_static()


def _write_files(tmp_path, n_files=3, per=20, seed=0):
    rs = np.random.RandomState(seed)
    w = np.array([0.5, -1.0, 2.0, 0.25])
    files = []
    for f in range(n_files):
        p = tmp_path / f"part-{f}.txt"
        with open(p, 'w') as fh:
            for _ in range(per):
                x = rs.randn(4)
                y = float(x @ w)
                fh.write(" ".join([str(v) for v in x]) + f"\t{y}\n")
        files.append(str(p))
    return files


GEN = r'''
import sys
sys.path.insert(0, {root!r})
import paddle.distributed.fleet as fleet

class Gen(fleet.MultiSlotDataGenerator):
    def generate_sample(self, line):
        def it():
            feats, y = line.rstrip('\n').split('\t')
            yield [('x', [float(v) for v in feats.split()]), ('y', [float(y)])]
        return it

Gen().run_from_stdin()
'''


def _slot_files(tmp_path, files):
    """The MultiSlot form of the raw files (what the generator script emits), for 'cat' pipes."""
    out = []
    for f in files:
        p = f + '.slots'
        with open(f) as fi, open(p, 'w') as fo:
            for line in fi:
                feats, y = line.rstrip('\n').split('\t')
                fo.write(f"4 {feats} 1 {y}\n")
        out.append(p)
    return out


@pytest.mark.parametrize('kind', ['InMemoryDataset', 'QueueDataset'])
def test_train_from_dataset(static_mode, tmp_path, kind):
    files = _write_files(tmp_path)
    gen = tmp_path / 'gen.py'
    gen.write_text(GEN.format(root=os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    # InMemoryDataset parses through the generator script once; QueueDataset re-reads every epoch,
    # so it streams the pre-formatted slot files through 'cat'
    pipe = f"{sys.executable} {gen}" if kind == 'InMemoryDataset' else 'cat'
    if kind == 'QueueDataset':
        files = _slot_files(tmp_path, files)
    main, start = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(main, start):
        x = paddle.static.data('x', [None, 4], 'float32')
        y = paddle.static.data('y', [None, 1], 'float32')
        fc = paddle.nn.Linear(4, 1)
        loss = paddle.mean(paddle.square(fc(x) - y))
        paddle.optimizer.SGD(0.05, parameters=fc.parameters()).minimize(loss)
    ds = paddle.distributed.InMemoryDataset() if kind == 'InMemoryDataset' else paddle.distributed.QueueDataset()
    ds.init(batch_size=8, thread_num=2, use_var=[x, y], pipe_command=pipe)
    ds.set_filelist(files)
    if kind == 'InMemoryDataset':
        ds.load_into_memory()
        assert ds.get_memory_data_size() == 60
        ds.local_shuffle()
        ds.global_shuffle()  # single process: a local shuffle
    exe = paddle.static.Executor()
    first = None

    class H:
        seen = []

        def handler(self, d):
            H.seen.append(float(d['loss']))
    for epoch in range(15):
        out = exe.train_from_dataset(main, ds, fetch_list=[loss], fetch_info=['loss'], print_period=1000,
                                     fetch_handler=H() if epoch == 0 else None)
        if first is None:
            first = float(out[0])
    assert len(H.seen) == 8  # ceil(60 / 8) batches in the first epoch
    assert float(out[0]) < 0.2 * first
    if kind == 'InMemoryDataset':
        ds.release_memory()
        assert ds.get_memory_data_size() == 0
    else:
        with pytest.raises(NotImplementedError):
            ds.local_shuffle()


def test_slot_parsing_errors_and_lod(tmp_path, static_mode):
    p = tmp_path / 'd.txt'
    p.write_text("2 1 2 1 7\n3 4 5 6 1 8\n")
    main = paddle.static.Program()
    with paddle.static.program_guard(main, paddle.static.Program()):
        ids = paddle.static.data('ids', [None, 1], 'int64', lod_level=1)
        lab = paddle.static.data('lab', [None, 1], 'int64')
    ds = paddle.distributed.QueueDataset()
    ds.init(batch_size=2, use_var=[ids, lab])
    ds.set_filelist([str(p)])
    feed = next(iter(ds._iter_batches()))
    assert feed['ids'].recursive_sequence_lengths() == [[2, 3]]
    np.testing.assert_array_equal(feed['ids'].numpy().reshape(-1), [1, 2, 4, 5, 6])
    np.testing.assert_array_equal(feed['lab'], [[7], [8]])
    bad = tmp_path / 'bad.txt'
    bad.write_text("2 1\n")
    ds.set_filelist([str(bad)])
    with pytest.raises(ValueError):
        next(iter(ds._iter_batches()))


def test_entry_attrs():
    from paddle.distributed import CountFilterEntry, ProbabilityEntry, ShowClickEntry
    assert ProbabilityEntry(0.1)._to_attr() == 'probability_entry:0.1'
    assert CountFilterEntry(10)._to_attr() == 'count_filter_entry:10'
    assert ShowClickEntry('show', 'click')._to_attr() == 'show_click_entry:show:click'
    with pytest.raises(ValueError):
        ProbabilityEntry(2.0)
