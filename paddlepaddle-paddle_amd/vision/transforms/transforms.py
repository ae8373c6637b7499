"""Transform classes (reference: python/paddle/vision/transforms/transforms.py — Compose:72,
BaseTransform:125, ToTensor:284 ... RandomErasing:1832).  ``keys`` lets one transform apply
consistently to ("image", "coords", ...) tuples, as in the reference."""
import math
import numbers
import random
from collections.abc import Sequence

import numpy as np

from . import functional as F
from ...core.tensor import Tensor


def _get_image_size(img):
    if F._is_pil_image(img):
        return img.size
    if isinstance(img, np.ndarray):
        return img.shape[:2][::-1]
    if isinstance(img, Tensor):
        return (img.shape[-1], img.shape[-2]) if img.ndim == 3 else (img.shape[1], img.shape[0])
    raise TypeError(f"Unexpected type {type(img)}")


class Compose:
    def __init__(self, transforms):
        self.transforms = list(transforms)

    def __call__(self, data):
        for t in self.transforms:
            data = t(data)
        return data

    def __repr__(self):
        return f"Compose({', '.join(type(t).__name__ for t in self.transforms)})"


class BaseTransform:
    def __init__(self, keys=None):
        if keys is None:
            keys = ("image",)
        elif not isinstance(keys, Sequence):
            raise ValueError(f"keys should be a sequence, but got keys={keys}")
        self.keys = keys
        self.params = None

    def _get_params(self, inputs):
        return None

    def __call__(self, inputs):
        if isinstance(inputs, tuple):
            self.params = self._get_params(inputs)
            outs = []
            for i, k in enumerate(self.keys):
                fn = getattr(self, f"_apply_{k}", None)
                outs.append(fn(inputs[i]) if fn is not None else inputs[i])
            outs.extend(inputs[len(self.keys):])
            return tuple(outs)
        self.params = self._get_params((inputs,))
        return self._apply_image(inputs)

    def _apply_image(self, image):
        raise NotImplementedError

    def _apply_boxes(self, boxes):
        return boxes

    def _apply_mask(self, mask):
        return self._apply_image(mask)


class ToTensor(BaseTransform):
    def __init__(self, data_format='CHW', keys=None):
        super().__init__(keys)
        self.data_format = data_format

    def _apply_image(self, img):
        return F.to_tensor(img, self.data_format)


class Resize(BaseTransform):
    def __init__(self, size, interpolation='bilinear', keys=None):
        super().__init__(keys)
        self.size, self.interpolation = size, interpolation

    def _apply_image(self, img):
        return F.resize(img, self.size, self.interpolation)


class RandomResizedCrop(BaseTransform):
    def __init__(self, size, scale=(0.08, 1.0), ratio=(3.0 / 4, 4.0 / 3), interpolation='bilinear', keys=None):
        super().__init__(keys)
        self.size = (size, size) if isinstance(size, int) else size
        self.scale, self.ratio, self.interpolation = scale, ratio, interpolation

    def _get_param(self, image, attempts=10):
        width, height = _get_image_size(image)
        area = height * width
        log_ratio = (math.log(self.ratio[0]), math.log(self.ratio[1]))
        for _ in range(attempts):
            target_area = random.uniform(*self.scale) * area
            aspect = math.exp(random.uniform(*log_ratio))
            w = int(round(math.sqrt(target_area * aspect)))
            h = int(round(math.sqrt(target_area / aspect)))
            if 0 < w <= width and 0 < h <= height:
                return random.randint(0, height - h), random.randint(0, width - w), h, w
        in_ratio = float(width) / float(height)
        if in_ratio < min(self.ratio):
            w, h = width, int(round(width / min(self.ratio)))
        elif in_ratio > max(self.ratio):
            h, w = height, int(round(height * max(self.ratio)))
        else:
            w, h = width, height
        return (height - h) // 2, (width - w) // 2, h, w

    def _apply_image(self, img):
        i, j, h, w = self._get_param(img)
        return F.resize(F.crop(img, i, j, h, w), self.size, self.interpolation)


class CenterCrop(BaseTransform):
    def __init__(self, size, keys=None):
        super().__init__(keys)
        self.size = size

    def _apply_image(self, img):
        return F.center_crop(img, self.size)


class RandomHorizontalFlip(BaseTransform):
    def __init__(self, prob=0.5, keys=None):
        super().__init__(keys)
        self.prob = prob

    def _get_params(self, inputs):
        return random.random() < self.prob

    def _apply_image(self, img):
        return F.hflip(img) if self.params else img


class RandomVerticalFlip(RandomHorizontalFlip):
    def _apply_image(self, img):
        return F.vflip(img) if self.params else img


class Normalize(BaseTransform):
    def __init__(self, mean=0.0, std=1.0, data_format='CHW', to_rgb=False, keys=None):
        super().__init__(keys)
        self.mean = [mean] * 3 if isinstance(mean, numbers.Number) else mean
        self.std = [std] * 3 if isinstance(std, numbers.Number) else std
        self.data_format, self.to_rgb = data_format, to_rgb

    def _apply_image(self, img):
        return F.normalize(img, self.mean, self.std, self.data_format, self.to_rgb)


class Transpose(BaseTransform):
    def __init__(self, order=(2, 0, 1), keys=None):
        super().__init__(keys)
        self.order = order

    def _apply_image(self, img):
        if isinstance(img, Tensor):
            return img.transpose(list(self.order))
        a = np.asarray(img)
        if a.ndim == 2:
            a = a[..., None]
        return a.transpose(self.order)


class BrightnessTransform(BaseTransform):
    def __init__(self, value, keys=None):
        super().__init__(keys)
        self.value = value

    def _apply_image(self, img):
        if self.value == 0:
            return img
        return F.adjust_brightness(img, random.uniform(max(0, 1 - self.value), 1 + self.value))


class ContrastTransform(BrightnessTransform):
    def _apply_image(self, img):
        if self.value == 0:
            return img
        return F.adjust_contrast(img, random.uniform(max(0, 1 - self.value), 1 + self.value))


class SaturationTransform(BrightnessTransform):
    def _apply_image(self, img):
        if self.value == 0:
            return img
        return F.adjust_saturation(img, random.uniform(max(0, 1 - self.value), 1 + self.value))


class HueTransform(BrightnessTransform):
    def _apply_image(self, img):
        if self.value == 0:
            return img
        return F.adjust_hue(img, random.uniform(-self.value, self.value))


class ColorJitter(BaseTransform):
    def __init__(self, brightness=0, contrast=0, saturation=0, hue=0, keys=None):
        super().__init__(keys)
        self.brightness, self.contrast, self.saturation, self.hue = brightness, contrast, saturation, hue

    def _apply_image(self, img):
        ts = []
        if self.brightness:
            ts.append(BrightnessTransform(self.brightness))
        if self.contrast:
            ts.append(ContrastTransform(self.contrast))
        if self.saturation:
            ts.append(SaturationTransform(self.saturation))
        if self.hue:
            ts.append(HueTransform(self.hue))
        random.shuffle(ts)
        for t in ts:
            img = t._apply_image(img)
        return img


class RandomCrop(BaseTransform):
    def __init__(self, size, padding=None, pad_if_needed=False, fill=0, padding_mode='constant', keys=None):
        super().__init__(keys)
        self.size = (int(size), int(size)) if isinstance(size, numbers.Number) else size
        self.padding, self.pad_if_needed, self.fill, self.padding_mode = padding, pad_if_needed, fill, padding_mode

    def _apply_image(self, img):
        if self.padding is not None:
            img = F.pad(img, self.padding, self.fill, self.padding_mode)
        w, h = _get_image_size(img)
        th, tw = self.size
        if self.pad_if_needed and w < tw:
            img = F.pad(img, (tw - w, 0), self.fill, self.padding_mode)
        if self.pad_if_needed and h < th:
            img = F.pad(img, (0, th - h), self.fill, self.padding_mode)
        w, h = _get_image_size(img)
        if w == tw and h == th:
            return img
        i, j = random.randint(0, h - th), random.randint(0, w - tw)
        return F.crop(img, i, j, th, tw)


class Pad(BaseTransform):
    def __init__(self, padding, fill=0, padding_mode='constant', keys=None):
        super().__init__(keys)
        self.padding, self.fill, self.padding_mode = padding, fill, padding_mode

    def _apply_image(self, img):
        return F.pad(img, self.padding, self.fill, self.padding_mode)


def _setup_angle(x, name, req_sizes=(2,)):
    if isinstance(x, numbers.Number):
        if x < 0:
            raise ValueError(f"If {name} is a single number, it must be positive.")
        return [-x, x]
    return [float(d) for d in x]


class RandomAffine(BaseTransform):
    def __init__(self, degrees, translate=None, scale=None, shear=None, interpolation='nearest', fill=0, center=None,
                 keys=None):
        super().__init__(keys)
        self.degrees = _setup_angle(degrees, 'degrees')
        self.translate, self.scale, self.interpolation, self.fill, self.center = translate, scale, interpolation, \
            fill, center
        self.shear = _setup_angle(shear, 'shear') if shear is not None else None

    def _apply_image(self, img):
        w, h = _get_image_size(img)
        angle = random.uniform(*self.degrees)
        tx = ty = 0
        if self.translate is not None:
            tx = int(round(random.uniform(-self.translate[0] * w, self.translate[0] * w)))
            ty = int(round(random.uniform(-self.translate[1] * h, self.translate[1] * h)))
        sc = random.uniform(*self.scale) if self.scale is not None else 1.0
        sh = [0.0, 0.0]
        if self.shear is not None:
            sh[0] = random.uniform(self.shear[0], self.shear[1])
            if len(self.shear) == 4:
                sh[1] = random.uniform(self.shear[2], self.shear[3])
        return F.affine(img, angle, (tx, ty), sc, sh, self.interpolation, self.fill, self.center)


class RandomRotation(BaseTransform):
    def __init__(self, degrees, interpolation='nearest', expand=False, center=None, fill=0, keys=None):
        super().__init__(keys)
        self.degrees = _setup_angle(degrees, 'degrees')
        self.interpolation, self.expand, self.center, self.fill = interpolation, expand, center, fill

    def _apply_image(self, img):
        return F.rotate(img, random.uniform(*self.degrees), self.interpolation, self.expand, self.center, self.fill)


class RandomPerspective(BaseTransform):
    def __init__(self, prob=0.5, distortion_scale=0.5, interpolation='nearest', fill=0, keys=None):
        super().__init__(keys)
        self.prob, self.distortion_scale, self.interpolation, self.fill = prob, distortion_scale, interpolation, fill

    def get_params(self, width, height, distortion_scale):
        hw, hh = width // 2, height // 2
        dw, dh = int(distortion_scale * hw), int(distortion_scale * hh)
        tl = [random.randint(0, dw), random.randint(0, dh)]
        tr = [width - 1 - random.randint(0, dw), random.randint(0, dh)]
        br = [width - 1 - random.randint(0, dw), height - 1 - random.randint(0, dh)]
        bl = [random.randint(0, dw), height - 1 - random.randint(0, dh)]
        start = [[0, 0], [width - 1, 0], [width - 1, height - 1], [0, height - 1]]
        return start, [tl, tr, br, bl]

    def _apply_image(self, img):
        if random.random() >= self.prob:
            return img
        w, h = _get_image_size(img)
        s, e = self.get_params(w, h, self.distortion_scale)
        return F.perspective(img, s, e, self.interpolation, self.fill)


class Grayscale(BaseTransform):
    def __init__(self, num_output_channels=1, keys=None):
        super().__init__(keys)
        self.num_output_channels = num_output_channels

    def _apply_image(self, img):
        return F.to_grayscale(img, self.num_output_channels)


class RandomErasing(BaseTransform):
    def __init__(self, prob=0.5, scale=(0.02, 0.33), ratio=(0.3, 3.3), value=0, inplace=False, keys=None):
        super().__init__(keys)
        self.prob, self.scale, self.ratio, self.value, self.inplace = prob, scale, ratio, value, inplace

    def _apply_image(self, img):
        if random.random() >= self.prob:
            return img
        w, h = _get_image_size(img)
        area = h * w
        for _ in range(10):
            ea = random.uniform(*self.scale) * area
            ar = math.exp(random.uniform(math.log(self.ratio[0]), math.log(self.ratio[1])))
            eh, ew = int(round(math.sqrt(ea * ar))), int(round(math.sqrt(ea / ar)))
            if eh < h and ew < w:
                i, j = random.randint(0, h - eh), random.randint(0, w - ew)
                v = self.value
                if v == 'random':
                    c = img.shape[0] if isinstance(img, Tensor) else (np.asarray(img).shape[2] if
                                                                     np.asarray(img).ndim == 3 else 1)
                    import torch
                    v = torch.randn(c, eh, ew)
                return F.erase(img, i, j, eh, ew, v, self.inplace)
        return img
