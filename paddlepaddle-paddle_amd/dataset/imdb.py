"""paddle.dataset.imdb: (word ids, label) readers over aclImdb_v1.tar.gz."""
from .common import local

__all__ = []


def _ds(mode, cutoff=150):
    from ..text.datasets import Imdb
    return Imdb(local('imdb', 'aclImdb_v1.tar.gz'), mode, cutoff)


def word_dict(cutoff=150):
    return _ds('train', cutoff).word_idx


def _reader(mode, word_idx):
    def reader():
        ds = _ds(mode)
        inv = {v: k for k, v in ds.word_idx.items()}
        unk = word_idx.get('<unk>', len(word_idx))
        for doc, lab in zip(ds.docs, ds.labels):
            yield [word_idx.get(inv[i], unk) for i in doc], lab
    return reader


def train(word_idx):
    return _reader('train', word_idx)


def test(word_idx):
    return _reader('test', word_idx)


def fetch():
    raise RuntimeError("fetch needs network access")
