"""paddle.dataset.voc2012: VOC2012 segmentation readers (image HWC uint8, class-index mask)."""
import numpy as np

from .common import local

__all__ = []


def reader_creator(filename, sub_name):
    def reader():
        from ..vision.datasets import VOC2012
        mode = {'trainval': 'train', 'train': 'test', 'val': 'valid'}[sub_name]
        ds = VOC2012(filename, mode=mode, backend='cv2')
        for i in range(len(ds)):
            img, lab = ds[i]
            yield np.asarray(img).astype('uint8'), np.asarray(lab)
    return reader


def train():
    return reader_creator(local('voc2012', 'VOCtrainval_11-May-2012.tar'), 'trainval')


def test():
    return reader_creator(local('voc2012', 'VOCtrainval_11-May-2012.tar'), 'train')


def val():
    return reader_creator(local('voc2012', 'VOCtrainval_11-May-2012.tar'), 'val')
