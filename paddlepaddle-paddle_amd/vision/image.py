"""paddle.vision.image (reference: python/paddle/vision/image.py)."""
_backend = ['pil']


def set_image_backend(backend):
    if backend not in ('pil', 'cv2', 'tensor'):
        raise ValueError(f"Expected backend are one of ['pil', 'cv2', 'tensor'], but got {backend}")
    if backend == 'cv2':
        raise ValueError("cv2 is not installed; use 'pil' or 'tensor'")
    _backend[0] = backend


def get_image_backend():
    return _backend[0]


def image_load(path, backend=None):
    backend = backend or _backend[0]
    from PIL import Image
    img = Image.open(path)
    if backend == 'tensor':
        from .transforms.functional import to_tensor
        return to_tensor(img.convert('RGB'))
    return img
