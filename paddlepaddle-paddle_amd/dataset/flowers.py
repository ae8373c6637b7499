"""paddle.dataset.flowers: Oxford 102 Flowers readers (102flowers.tgz, imagelabels.mat, setid.mat),
samples mapped by ``mapper`` (default: resize-short 256, crop 224, CHW float32, mean-subtracted)."""
import numpy as np

from .common import local
from . import image as _image

__all__ = []


def default_mapper(is_train, sample):
    img, label = sample
    img = _image.simple_transform(np.asarray(img), 256, 224, is_train, mean=[103.94, 116.78, 123.68])
    return img.flatten().astype('float32'), label


def train_mapper(sample):
    return default_mapper(True, sample)


def test_mapper(sample):
    return default_mapper(False, sample)


def reader_creator(mode, mapper, buffered_size=1024, use_xmap=True, cycle=False):
    def reader():
        from ..vision.datasets import Flowers
        ds = Flowers(local('flowers', '102flowers.tgz'), local('flowers', 'imagelabels.mat'),
                     local('flowers', 'setid.mat'), mode=mode, backend='cv2')
        while True:
            for i in range(len(ds)):
                img, lab = ds[i]
                yield mapper((img, int(lab[0]) - 1))
            if not cycle:
                break
    return reader


def train(mapper=train_mapper, buffered_size=1024, use_xmap=True, cycle=False):
    return reader_creator('train', mapper, buffered_size, use_xmap, cycle)


def test(mapper=test_mapper, buffered_size=1024, use_xmap=True, cycle=False):
    return reader_creator('test', mapper, buffered_size, use_xmap, cycle)


def valid(mapper=test_mapper, buffered_size=1024, use_xmap=True):
    return reader_creator('valid', mapper, buffered_size, use_xmap)


def fetch():
    raise RuntimeError("fetch needs network access")
