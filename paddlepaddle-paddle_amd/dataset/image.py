"""paddle.dataset.image: numpy/PIL image helpers of the legacy readers (reference:
python/paddle/dataset/image.py, cv2-based there; HWC arrays, BGR-free RGB here)."""
import io
import tarfile

import numpy as np

__all__ = []


def load_image_bytes(bytes, is_color=True):  # noqa: A002
    from PIL import Image
    im = Image.open(io.BytesIO(bytes))
    return np.asarray(im.convert('RGB' if is_color else 'L'))


def load_image(file, is_color=True):
    with open(file, 'rb') as f:
        return load_image_bytes(f.read(), is_color)


def resize_short(im, size):
    from PIL import Image
    h, w = im.shape[:2]
    if h > w:
        nh, nw = size * h // w, size
    else:
        nh, nw = size, size * w // h
    return np.asarray(Image.fromarray(im).resize((nw, nh), Image.BICUBIC))


def to_chw(im, order=(2, 0, 1)):
    assert len(im.shape) == len(order)
    return im.transpose(order)


def center_crop(im, size, is_color=True):
    h, w = im.shape[:2]
    h0, w0 = (h - size) // 2, (w - size) // 2
    return im[h0:h0 + size, w0:w0 + size]


def random_crop(im, size, is_color=True):
    h, w = im.shape[:2]
    h0, w0 = np.random.randint(0, h - size + 1), np.random.randint(0, w - size + 1)
    return im[h0:h0 + size, w0:w0 + size]


def left_right_flip(im, is_color=True):
    return im[:, ::-1]


def simple_transform(im, resize_size, crop_size, is_train, is_color=True, mean=None):
    im = resize_short(im, resize_size)
    if is_train:
        im = random_crop(im, crop_size, is_color)
        if np.random.randint(2) == 0:
            im = left_right_flip(im, is_color)
    else:
        im = center_crop(im, crop_size, is_color)
    if im.ndim == 3:
        im = to_chw(im)
    im = im.astype('float32')
    if mean is not None:
        mean = np.array(mean, dtype=np.float32)
        if mean.ndim == 1 and is_color:
            mean = mean[:, np.newaxis, np.newaxis]
        im -= mean
    return im


def load_and_transform(filename, resize_size, crop_size, is_train, is_color=True, mean=None):
    return simple_transform(load_image(filename, is_color), resize_size, crop_size, is_train, is_color, mean)


def batch_images_from_tar(data_file, dataset_name, img2label, num_per_batch=1024):
    """Group the tar's images into lists of (raw bytes, label) of ``num_per_batch`` entries;
    returns the list of batches (the reference pickles them to disk; nothing is written here)."""
    batches, cur = [], []
    with tarfile.open(data_file) as tf:
        for m in tf.getmembers():
            if m.name in img2label:
                cur.append((tf.extractfile(m).read(), img2label[m.name]))
                if len(cur) == num_per_batch:
                    batches.append(cur)
                    cur = []
    if cur:
        batches.append(cur)
    return batches
