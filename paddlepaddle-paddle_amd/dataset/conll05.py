"""paddle.dataset.conll05: CoNLL-05 SRL test reader, dictionaries and embedding path."""
from .common import local

__all__ = []


def _ds():
    from ..text.datasets import Conll05st
    return Conll05st(local('conll05st', 'conll05st-tests.tar.gz'), local('conll05st', 'wordDict.txt'),
                     local('conll05st', 'verbDict.txt'), local('conll05st', 'targetDict.txt'),
                     local('conll05st', 'emb'))


def get_dict():
    return _ds().get_dict()


def get_embedding():
    return local('conll05st', 'emb')


def test():
    def reader():
        ds = _ds()
        for i in range(len(ds)):
            yield tuple(x.tolist() for x in ds[i])
    return reader


def fetch():
    raise RuntimeError("fetch needs network access")
