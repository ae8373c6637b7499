"""paddle.dataset.uci_housing: (13 normalised features, [price]) readers from housing.data."""
from .common import local

__all__ = []

feature_names = ['CRIM', 'ZN', 'INDUS', 'CHAS', 'NOX', 'RM', 'AGE', 'DIS', 'RAD', 'TAX', 'PTRATIO', 'B', 'LSTAT']


def _reader(mode, data_file=None):
    def reader():
        from ..text.datasets import UCIHousing
        ds = UCIHousing(data_file or local('uci_housing', 'housing.data'), mode)
        for i in range(len(ds)):
            yield ds[i]
    return reader


def train(data_file=None):
    return _reader('train', data_file)


def test(data_file=None):
    return _reader('test', data_file)


def fetch():
    raise RuntimeError("fetch needs network access")
