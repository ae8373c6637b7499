"""paddle.dataset.cifar: (3072 float32 pixels / 255, int label) readers, read from the BINARY
CIFAR distributions (cifar-10-binary.tar.gz / cifar-100-binary.tar.gz) — the python-pickle
tarballs are never unpickled."""
from .common import local

__all__ = []


def reader_creator(filename, sub_name=None, cycle=False, hundred=False):
    def reader():
        from ..vision.datasets import Cifar10, Cifar100
        ds = (Cifar100 if hundred else Cifar10)(filename, mode=sub_name or 'train', backend='cv2')
        while True:
            for i in range(len(ds)):
                yield ds.data[i].transpose(2, 0, 1).reshape(-1).astype('float32') / 255.0, int(ds.labels[i])
            if not cycle:
                break
    return reader


def train100():
    return reader_creator(local('cifar', 'cifar-100-binary.tar.gz'), 'train', hundred=True)


def test100():
    return reader_creator(local('cifar', 'cifar-100-binary.tar.gz'), 'test', hundred=True)


def train10(cycle=False):
    return reader_creator(local('cifar', 'cifar-10-binary.tar.gz'), 'train', cycle)


def test10(cycle=False):
    return reader_creator(local('cifar', 'cifar-10-binary.tar.gz'), 'test', cycle)


def fetch():
    raise RuntimeError("fetch needs network access")
