"""paddle.dataset.imikolov: PTB n-gram / sequence readers over simple-examples.tgz."""
from .common import local

__all__ = []


class DataType:
    NGRAM = 1
    SEQ = 2


def _file():
    return local('imikolov', 'simple-examples.tgz')


def build_dict(min_word_freq=50):
    from ..text.datasets import Imikolov
    return Imikolov(_file(), 'NGRAM', 2, 'train', min_word_freq).word_idx


def _reader(mode, word_idx, n, data_type):
    def reader():
        from ..text.datasets import Imikolov
        ds = Imikolov(_file(), 'NGRAM' if data_type == DataType.NGRAM else 'SEQ', n, mode)
        inv = {v: k for k, v in ds.word_idx.items()}
        unk = word_idx['<unk>']
        remap = lambda ids: [word_idx.get(inv[i], unk) for i in ids]  # noqa: E731
        for sample in ds.data:
            if data_type == DataType.NGRAM:
                yield tuple(remap(sample))
            else:
                yield remap(sample[0]), remap(sample[1])
    return reader


def train(word_idx, n, data_type=DataType.NGRAM):
    return _reader('train', word_idx, n, data_type)


def test(word_idx, n, data_type=DataType.NGRAM):
    return _reader('test', word_idx, n, data_type)


def fetch():
    raise RuntimeError("fetch needs network access")
