"""paddle.dataset.wmt16: Multi30k en-de translation readers over wmt16.tar.gz."""
from .common import local

__all__ = []


def _ds(mode, src_dict_size, trg_dict_size, src_lang):
    from ..text.datasets import WMT16
    return WMT16(local('wmt16', 'wmt16.tar.gz'), mode, src_dict_size, trg_dict_size, src_lang)


def _reader(mode, src_dict_size, trg_dict_size, src_lang):
    def reader():
        ds = _ds(mode, src_dict_size, trg_dict_size, src_lang)
        yield from zip(ds.src_ids, ds.trg_ids, ds.trg_ids_next)
    return reader


def train(src_dict_size, trg_dict_size, src_lang="en"):
    return _reader('train', src_dict_size, trg_dict_size, src_lang)


def test(src_dict_size, trg_dict_size, src_lang="en"):
    return _reader('test', src_dict_size, trg_dict_size, src_lang)


def validation(src_dict_size, trg_dict_size, src_lang="en"):
    return _reader('val', src_dict_size, trg_dict_size, src_lang)


def get_dict(lang, dict_size, reverse=False):
    other = 'de' if lang == 'en' else 'en'
    return _ds('train', dict_size, dict_size, lang).get_dict(lang, reverse) if lang in ('en', 'de') else \
        _ds('train', dict_size, dict_size, other).get_dict(lang, reverse)


def fetch():
    raise RuntimeError("fetch needs network access")
