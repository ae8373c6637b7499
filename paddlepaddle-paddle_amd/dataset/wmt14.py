"""paddle.dataset.wmt14: en-fr (shrinked) translation readers over wmt_shrinked_data.tgz."""
from .common import local

__all__ = []


def _ds(mode, dict_size):
    from ..text.datasets import WMT14
    return WMT14(local('wmt14', 'wmt_shrinked_data.tgz'), mode, dict_size)


def _reader(mode, dict_size):
    def reader():
        ds = _ds(mode, dict_size)
        yield from zip(ds.src_ids, ds.trg_ids, ds.trg_ids_next)
    return reader


def train(dict_size):
    return _reader('train', dict_size)


def test(dict_size):
    return _reader('test', dict_size)


def gen(dict_size):
    return _reader('gen', dict_size)


def get_dict(dict_size, reverse=True):
    return _ds('train', dict_size).get_dict(reverse)


def fetch():
    raise RuntimeError("fetch needs network access")
