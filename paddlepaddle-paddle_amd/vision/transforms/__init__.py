"""paddle.vision.transforms (reference: python/paddle/vision/transforms/__init__.py)."""
from .transforms import (BaseTransform, Compose, Resize, RandomResizedCrop, CenterCrop,  # noqa: F401
                         RandomHorizontalFlip, RandomVerticalFlip, Transpose, Normalize, BrightnessTransform,
                         SaturationTransform, ContrastTransform, HueTransform, ColorJitter, RandomCrop, Pad,
                         RandomAffine, RandomRotation, RandomPerspective, Grayscale, ToTensor, RandomErasing)
from .functional import (to_tensor, hflip, vflip, resize, pad, affine, rotate, perspective,  # noqa: F401
                         to_grayscale, crop, center_crop, adjust_brightness, adjust_contrast, adjust_hue,
                         adjust_saturation, normalize, erase)
from . import functional  # noqa: F401
