"""paddle.dataset.mnist: (784 float32 pixels scaled to [-1, 1], int label) readers."""
from .common import local

__all__ = []

_FILES = {'train': ('train-images-idx3-ubyte.gz', 'train-labels-idx1-ubyte.gz'),
          'test': ('t10k-images-idx3-ubyte.gz', 't10k-labels-idx1-ubyte.gz')}


def reader_creator(image_filename, label_filename, buffer_size=100):
    def reader():
        from ..vision.datasets import MNIST
        ds = MNIST(image_filename, label_filename, backend='cv2')
        imgs = ds.images.reshape(len(ds), -1).astype('float32') / 255.0 * 2.0 - 1.0
        for i in range(len(ds)):
            yield imgs[i], int(ds.labels[i])
    return reader


def _split(mode):
    img, lab = _FILES[mode]
    return reader_creator(local('mnist', img), local('mnist', lab))


def train():
    return _split('train')


def test():
    return _split('test')


def fetch():
    raise RuntimeError("fetch needs network access")

