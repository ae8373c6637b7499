"""paddle.dataset.movielens: MovieLens-1M rating readers and metadata over ml-1m.zip."""
from .common import local

__all__ = []
_cache = {}


def _ds(mode='train'):
    if mode not in _cache:
        from ..text.datasets import Movielens
        _cache[mode] = Movielens(local('movielens', 'ml-1m.zip'), mode)
    return _cache[mode]


def _reader(mode):
    def reader():
        for sample in _ds(mode).data:
            yield sample
    return reader


def train():
    return _reader('train')


def test():
    return _reader('test')


def get_movie_title_dict():
    return _ds().movie_title_dict


def movie_categories():
    return _ds().categories_dict


def max_movie_id():
    return max(_ds().movie_info)


def max_user_id():
    return max(_ds().user_info)


def max_job_id():
    return max(u.job_id for u in _ds().user_info.values())


def user_info():
    return _ds().user_info


def movie_info():
    return _ds().movie_info


def fetch():
    raise RuntimeError("fetch needs network access")
