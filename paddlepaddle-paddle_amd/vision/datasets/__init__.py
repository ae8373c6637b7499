"""paddle.vision.datasets (reference: python/paddle/vision/datasets/{mnist,cifar,flowers,voc2012,
folder}.py).

No network here: every dataset reads local files (``image_path``/``label_path``/``data_file``;
``download=True`` raises).  CIFAR is read from the *binary* distribution (``*.bin`` batches or
their tar.gz), never by unpickling.  ``DatasetFolder``/``ImageFolder`` scan a directory tree.
"""
import gzip
import os
import struct
import tarfile

import numpy as np

from ...io import Dataset

IMG_EXTENSIONS = ('.jpg', '.jpeg', '.png', '.ppm', '.bmp', '.pgm', '.tif', '.tiff', '.webp')


def _no_download(name):
    raise RuntimeError(f"{name}: download is not possible (no network); pass local file paths")


def _open(path):
    return gzip.open(path, 'rb') if str(path).endswith('.gz') else open(path, 'rb')


class MNIST(Dataset):
    NAME = 'mnist'

    def __init__(self, image_path=None, label_path=None, mode='train', transform=None, download=True,
                 backend=None):
        if image_path is None or label_path is None:
            _no_download(type(self).__name__)
        self.mode, self.transform, self.backend = mode.lower(), transform, backend or 'pil'
        with _open(image_path) as f:
            magic, n, rows, cols = struct.unpack('>IIII', f.read(16))
            self.images = np.frombuffer(f.read(), dtype=np.uint8).reshape(n, rows, cols)
        with _open(label_path) as f:
            magic, n = struct.unpack('>II', f.read(8))
            self.labels = np.frombuffer(f.read(), dtype=np.uint8).astype(np.int64)

    def __getitem__(self, idx):
        image, label = self.images[idx], np.array([self.labels[idx]], dtype=np.int64)
        if self.backend == 'pil':
            from PIL import Image
            image = Image.fromarray(image, mode='L')
        else:
            image = image.astype(np.float32)
        if self.transform is not None:
            image = self.transform(image)
        return image, label

    def __len__(self):
        return len(self.labels)


class FashionMNIST(MNIST):
    NAME = 'fashion-mnist'


class Cifar10(Dataset):
    _n_label_bytes = 1

    def __init__(self, data_file=None, mode='train', transform=None, download=True, backend=None):
        if data_file is None:
            _no_download(type(self).__name__)
        self.mode, self.transform, self.backend = mode.lower(), transform, backend or 'pil'
        blobs = []
        if os.path.isdir(data_file):
            for fn in sorted(os.listdir(data_file)):
                if self._want(fn):
                    with open(os.path.join(data_file, fn), 'rb') as f:
                        blobs.append(f.read())
        else:
            with tarfile.open(data_file) as tf:
                for m in sorted(tf.getmembers(), key=lambda m: m.name):
                    if m.isfile() and self._want(os.path.basename(m.name)):
                        blobs.append(tf.extractfile(m).read())
        rec = self._n_label_bytes + 3072
        data = np.frombuffer(b''.join(blobs), dtype=np.uint8).reshape(-1, rec)
        self.labels = data[:, self._n_label_bytes - 1].astype(np.int64)
        self.data = data[:, self._n_label_bytes:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1)

    def _want(self, fn):
        if not fn.endswith('.bin'):
            return False
        return ('test' in fn) == (self.mode == 'test')

    def __getitem__(self, idx):
        image, label = self.data[idx], np.array(self.labels[idx], dtype=np.int64)
        if self.backend == 'pil':
            from PIL import Image
            image = Image.fromarray(image)
        if self.transform is not None:
            image = self.transform(image)
        return image, label

    def __len__(self):
        return len(self.labels)


class Cifar100(Cifar10):
    _n_label_bytes = 2  # coarse, fine: the fine label is used


def has_valid_extension(filename, extensions):
    return filename.lower().endswith(tuple(extensions))


def default_loader(path):
    from PIL import Image
    with open(path, 'rb') as f:
        return Image.open(f).convert('RGB')


class DatasetFolder(Dataset):
    def __init__(self, root, loader=None, extensions=None, transform=None, is_valid_file=None):
        self.root = root
        self.transform = transform
        extensions = IMG_EXTENSIONS if extensions is None and is_valid_file is None else extensions
        classes = sorted(d.name for d in os.scandir(root) if d.is_dir())
        self.classes = classes
        self.class_to_idx = {c: i for i, c in enumerate(classes)}
        samples = []
        for c in classes:
            for dp, _, fns in sorted(os.walk(os.path.join(root, c))):
                for fn in sorted(fns):
                    p = os.path.join(dp, fn)
                    ok = is_valid_file(p) if is_valid_file is not None else has_valid_extension(fn, extensions)
                    if ok:
                        samples.append((p, self.class_to_idx[c]))
        if not samples:
            raise RuntimeError(f"Found 0 files in subfolders of: {root}")
        self.samples = samples
        self.targets = [s[1] for s in samples]
        self.loader = loader or default_loader

    def __getitem__(self, index):
        path, target = self.samples[index]
        sample = self.loader(path)
        if self.transform is not None:
            sample = self.transform(sample)
        return sample, np.array([target], dtype=np.int64)

    def __len__(self):
        return len(self.samples)


class ImageFolder(Dataset):
    """Flat folder of images (no labels)."""

    def __init__(self, root, loader=None, extensions=None, transform=None, is_valid_file=None):
        self.root = root
        extensions = IMG_EXTENSIONS if extensions is None and is_valid_file is None else extensions
        samples = []
        for dp, _, fns in sorted(os.walk(root)):
            for fn in sorted(fns):
                p = os.path.join(dp, fn)
                ok = is_valid_file(p) if is_valid_file is not None else has_valid_extension(fn, extensions)
                if ok:
                    samples.append(p)
        if not samples:
            raise RuntimeError(f"Found 0 files in: {root}")
        self.samples = samples
        self.loader = loader or default_loader
        self.transform = transform

    def __getitem__(self, index):
        sample = self.loader(self.samples[index])
        if self.transform is not None:
            sample = self.transform(sample)
        return [sample]

    def __len__(self):
        return len(self.samples)


def _backend(backend):
    if backend is None:
        from ..image import get_image_backend
        backend = get_image_backend()
    if backend not in ('pil', 'cv2'):
        raise ValueError(f"Expected backend are one of ['pil', 'cv2'], but got {backend}")
    return backend


class Flowers(Dataset):
    """Oxford 102 Flowers from the published files: ``102flowers.tgz`` (jpg/image_NNNNN.jpg; read
    in place, not extracted), ``imagelabels.mat`` and ``setid.mat`` (scipy.io.loadmat: MATLAB
    arrays, nothing executed).  As the reference, 'train' uses the large 'tstid' split and
    'test' the small 'trnid' one."""

    _FLAG = {'train': 'tstid', 'test': 'trnid', 'valid': 'valid'}

    def __init__(self, data_file=None, label_file=None, setid_file=None, mode='train', transform=None,
                 download=True, backend=None):
        m = mode.lower()
        assert m in self._FLAG, f"mode should be 'train', 'valid' or 'test', but got {mode}"
        if not data_file or not label_file or not setid_file:
            _no_download('Flowers')
        self.backend, self.transform = _backend(backend), transform
        import scipy.io as scio
        self.labels = scio.loadmat(label_file)['labels'][0]
        self.indexes = scio.loadmat(setid_file)[self._FLAG[m]][0]
        self.data_file = data_file
        self._tar = None

    def _image_bytes(self, name):
        if os.path.isdir(self.data_file):
            with open(os.path.join(self.data_file, name), 'rb') as f:
                return f.read()
        if self._tar is None:
            self._tar = tarfile.open(self.data_file)
            self._members = {m.name.lstrip('./'): m for m in self._tar.getmembers()}
        return self._tar.extractfile(self._members[name]).read()

    def __getitem__(self, idx):
        import io as _io
        from PIL import Image
        index = int(self.indexes[idx])
        label = np.array([self.labels[index - 1]]).astype('int64')
        image = Image.open(_io.BytesIO(self._image_bytes("jpg/image_%05d.jpg" % index)))
        if self.backend == 'cv2':
            image = np.array(image)
        if self.transform is not None:
            image = self.transform(image)
        if self.backend == 'cv2':
            image = np.asarray(image).astype('float32')
        return image, label

    def __len__(self):
        return len(self.indexes)

    def __getstate__(self):
        d = dict(self.__dict__)
        d['_tar'] = None  # reopened lazily in each worker
        return d


class VOC2012(Dataset):
    """PASCAL VOC2012 segmentation from ``VOCtrainval_11-May-2012.tar`` (or its extracted root):
    (image, class-index mask).  Split map as the reference: train -> trainval, test -> train,
    valid -> val."""

    _FLAG = {'train': 'trainval', 'test': 'train', 'valid': 'val'}
    _SET, _IMG, _LAB = ('VOCdevkit/VOC2012/ImageSets/Segmentation/{}.txt', 'VOCdevkit/VOC2012/JPEGImages/{}.jpg',
                        'VOCdevkit/VOC2012/SegmentationClass/{}.png')

    def __init__(self, data_file=None, mode='train', transform=None, download=True, backend=None):
        m = mode.lower()
        assert m in self._FLAG, f"mode should be 'train', 'valid' or 'test', but got {mode}"
        if data_file is None:
            _no_download('VOC2012')
        self.backend, self.transform, self.data_file = _backend(backend), transform, data_file
        self._tar = None
        ids = self._read(self._SET.format(self._FLAG[m])).decode('utf-8').split()
        self.data = [self._IMG.format(i) for i in ids]
        self.labels = [self._LAB.format(i) for i in ids]

    def _read(self, name):
        if os.path.isdir(self.data_file):
            root = self.data_file
            if not os.path.exists(os.path.join(root, name)) and name.startswith('VOCdevkit/VOC2012/'):
                name = name[len('VOCdevkit/VOC2012/'):]  # the extracted VOC2012 directory itself
            with open(os.path.join(root, name), 'rb') as f:
                return f.read()
        if self._tar is None:
            self._tar = tarfile.open(self.data_file)
            self._members = {mm.name: mm for mm in self._tar.getmembers()}
        return self._tar.extractfile(self._members[name]).read()

    def __getitem__(self, idx):
        import io as _io
        from PIL import Image
        img = Image.open(_io.BytesIO(self._read(self.data[idx])))
        lab = Image.open(_io.BytesIO(self._read(self.labels[idx])))
        if self.backend == 'cv2':
            img, lab = np.array(img), np.array(lab)
        if self.transform is not None:
            img = self.transform(img)
        if self.backend == 'cv2':
            return np.asarray(img).astype('float32'), np.asarray(lab)
        return img, np.array(lab)

    def __len__(self):
        return len(self.data)

    def __getstate__(self):
        d = dict(self.__dict__)
        d['_tar'] = None
        return d


__all__ = ['DatasetFolder', 'ImageFolder', 'MNIST', 'FashionMNIST', 'Flowers', 'Cifar10', 'Cifar100', 'VOC2012']
