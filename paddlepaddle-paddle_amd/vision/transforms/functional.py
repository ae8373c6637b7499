"""paddle.vision.transforms.functional (reference: python/paddle/vision/transforms/functional.py
and its pil/cv2/tensor backends).

One implementation on torch tensors: PIL images and HWC numpy arrays are converted to a CHW
tensor, transformed, and converted back to the caller's type; paddle Tensors (CHW) stay on their
device, so batched GPU augmentation works the same way.
"""
import math
import numbers

import numpy as np
import torch
import torch.nn.functional as TF

from ...core.tensor import Tensor, _wrap, _unwrap

try:
    from PIL import Image
except ImportError:  # pragma: no cover
    Image = None


def _is_pil_image(img):
    return Image is not None and isinstance(img, Image.Image)


def _is_tensor_image(img):
    return isinstance(img, Tensor) and img.ndim in (2, 3)


def _is_numpy_image(img):
    return isinstance(img, np.ndarray) and img.ndim in (2, 3)


def _in(img, data_format='CHW'):
    """→ (CHW torch tensor, restore fn)."""
    if _is_pil_image(img):
        mode = img.mode
        a = np.array(img)
        t = torch.from_numpy(a.copy())
        t = t.unsqueeze(0) if t.dim() == 2 else t.permute(2, 0, 1)

        def back(o):
            o = o.clamp(0, 255).round().to(torch.uint8) if o.is_floating_point() else o
            arr = o[0].numpy() if o.shape[0] == 1 else o.permute(1, 2, 0).numpy()
            return Image.fromarray(arr, mode if (o.shape[0] == len(mode) or mode in ('L', 'P')) and mode != 'P'
                                   else None)
        return t, back
    if isinstance(img, np.ndarray):
        t = torch.from_numpy(np.ascontiguousarray(img))
        two = t.dim() == 2
        t = t.unsqueeze(0) if two else t.permute(2, 0, 1)
        dt = img.dtype

        def back(o):
            if dt == np.uint8 and o.is_floating_point():
                o = o.clamp(0, 255).round().to(torch.uint8)
            a = o[0] if two and o.shape[0] == 1 else o.permute(1, 2, 0)
            return a.numpy().astype(dt, copy=False)
        return t, back
    if isinstance(img, Tensor):
        t = img._t
        hwc = data_format.upper() == 'HWC'
        two = t.dim() == 2
        t = t.unsqueeze(0) if two else (t.permute(2, 0, 1) if hwc else t)

        def back(o):
            o = o[0] if two else (o.permute(1, 2, 0) if hwc else o)
            return _wrap(o)
        return t, back
    if isinstance(img, torch.Tensor):
        return img, lambda o: o
    raise TypeError(f"img should be PIL Image, ndarray or Tensor, got {type(img)}")


def _size_hw(t):
    return t.shape[-2], t.shape[-1]


def to_tensor(pic, data_format='CHW'):
    if _is_pil_image(pic) or isinstance(pic, np.ndarray):
        a = np.array(pic) if _is_pil_image(pic) else pic
        if a.ndim == 2:
            a = a[:, :, None]
        t = torch.from_numpy(np.ascontiguousarray(a))
        t = t.float().div(255.0) if a.dtype == np.uint8 else t.float()
        if data_format.upper() == 'CHW':
            t = t.permute(2, 0, 1)
        return _wrap(t.contiguous())
    if isinstance(pic, Tensor):
        return pic if data_format.upper() == 'CHW' else _wrap(pic._t.permute(1, 2, 0))
    raise TypeError(f"pic should be PIL Image, ndarray or Tensor, got {type(pic)}")


_MODES = {'nearest': 'nearest', 'bilinear': 'bilinear', 'bicubic': 'bicubic', 'area': 'area', 'lanczos': 'bicubic'}


def resize(img, size, interpolation='bilinear'):
    t, back = _in(img)
    h, w = _size_hw(t)
    if isinstance(size, int):
        if (w <= h and w == size) or (h <= w and h == size):
            return img
        if w < h:
            ow, oh = size, int(size * h / w)
        else:
            oh, ow = size, int(size * w / h)
    else:
        oh, ow = size
    mode = _MODES.get(interpolation, 'bilinear')
    x = t.unsqueeze(0).float()
    kw = {'align_corners': False} if mode in ('bilinear', 'bicubic') else {}
    if mode in ('bilinear', 'bicubic') and (oh < h or ow < w):
        kw['antialias'] = True
    out = TF.interpolate(x, size=(oh, ow), mode=mode, **kw)[0]
    if not t.is_floating_point():
        out = out.clamp(0, 255).round().to(t.dtype)
    return back(out)


def pad(img, padding, fill=0, padding_mode='constant'):
    t, back = _in(img)
    if isinstance(padding, int):
        pl = pr = pt = pb = padding
    elif len(padding) == 2:
        pl, pt = padding
        pr, pb = padding
    else:
        pl, pt, pr, pb = padding
    mode = {'constant': 'constant', 'edge': 'replicate', 'reflect': 'reflect', 'symmetric': 'reflect'}[padding_mode]
    x = t.unsqueeze(0)
    if mode == 'constant':
        out = TF.pad(x.float() if not x.is_floating_point() else x, (pl, pr, pt, pb), value=float(fill)
                     if isinstance(fill, numbers.Number) else 0.0)
        if isinstance(fill, (tuple, list)):
            for c, v in enumerate(fill[:out.shape[1]]):
                ch = out[0, c]
                mask = torch.ones_like(ch, dtype=torch.bool)
                mask[pt:pt + t.shape[1], pl:pl + t.shape[2]] = False
                ch[mask] = float(v)
    else:
        if padding_mode == 'symmetric':
            x2 = torch.cat([x[..., :, :pl].flip(-1), x, x[..., :, x.shape[-1] - pr:].flip(-1)], -1) if (pl or pr) \
                else x
            out = torch.cat([x2[..., :pt, :].flip(-2), x2, x2[..., x2.shape[-2] - pb:, :].flip(-2)], -2) if (pt or pb) \
                else x2
        else:
            out = TF.pad(x.float(), (pl, pr, pt, pb), mode=mode)
    out = out[0]
    if not t.is_floating_point():
        out = out.round().to(t.dtype)
    return back(out)


def crop(img, top, left, height, width):
    t, back = _in(img)
    return back(t[:, top:top + height, left:left + width])


def center_crop(img, output_size):
    t, back = _in(img)
    if isinstance(output_size, int):
        output_size = (output_size, output_size)
    h, w = _size_hw(t)
    th, tw = output_size
    i = int(round((h - th) / 2.0))
    j = int(round((w - tw) / 2.0))
    return back(t[:, i:i + th, j:j + tw])


def hflip(img):
    t, back = _in(img)
    return back(t.flip(-1))


def vflip(img):
    t, back = _in(img)
    return back(t.flip(-2))


def _blend(a, b, ratio, is_float):
    bound = 1.0 if is_float else 255.0
    return (ratio * a + (1.0 - ratio) * b).clamp(0, bound)


def _gray(t):
    f = t.float()
    if t.shape[0] == 1:
        return f
    return (0.299 * f[0] + 0.587 * f[1] + 0.114 * f[2]).unsqueeze(0)


def adjust_brightness(img, brightness_factor):
    t, back = _in(img)
    f = t.float()
    out = _blend(f, torch.zeros_like(f), brightness_factor, t.is_floating_point())
    return back(out if t.is_floating_point() else out.round().to(t.dtype))


def adjust_contrast(img, contrast_factor):
    t, back = _in(img)
    f = t.float()
    mean = _gray(t).mean()
    out = _blend(f, mean.expand_as(f), contrast_factor, t.is_floating_point())
    return back(out if t.is_floating_point() else out.round().to(t.dtype))


def adjust_saturation(img, saturation_factor):
    t, back = _in(img)
    f = t.float()
    out = _blend(f, _gray(t).expand_as(f), saturation_factor, t.is_floating_point())
    return back(out if t.is_floating_point() else out.round().to(t.dtype))


def _rgb2hsv(img):
    r, g, b = img.unbind(0)
    maxc, _ = img.max(0)
    minc, _ = img.min(0)
    eqc = maxc == minc
    cr = maxc - minc
    ones = torch.ones_like(maxc)
    s = cr / torch.where(eqc, ones, maxc)
    cr_div = torch.where(eqc, ones, cr)
    rc, gc, bc = (maxc - r) / cr_div, (maxc - g) / cr_div, (maxc - b) / cr_div
    hr = (maxc == r) * (bc - gc)
    hg = ((maxc == g) & (maxc != r)) * (2.0 + rc - bc)
    hb = ((maxc != g) & (maxc != r)) * (4.0 + gc - rc)
    h = torch.fmod((hr + hg + hb) / 6.0 + 1.0, 1.0)
    return torch.stack((h, s, maxc))


def _hsv2rgb(img):
    h, s, v = img.unbind(0)
    i = torch.floor(h * 6.0)
    f = h * 6.0 - i
    i = i.to(torch.int32) % 6
    p = (v * (1.0 - s)).clamp(0.0, 1.0)
    q = (v * (1.0 - s * f)).clamp(0.0, 1.0)
    t = (v * (1.0 - s * (1.0 - f))).clamp(0.0, 1.0)
    mask = i.unsqueeze(0) == torch.arange(6, device=i.device).view(-1, 1, 1)
    a1 = torch.stack((v, q, p, p, t, v))
    a2 = torch.stack((t, v, v, q, p, p))
    a3 = torch.stack((p, p, t, v, v, q))
    a4 = torch.stack((a1, a2, a3))
    return torch.einsum("ijk, xijk -> xjk", mask.to(img.dtype), a4)


def adjust_hue(img, hue_factor):
    if not -0.5 <= hue_factor <= 0.5:
        raise ValueError(f"hue_factor ({hue_factor}) is not in [-0.5, 0.5].")
    t, back = _in(img)
    if t.shape[0] == 1:
        return img
    f = t.float() / (1.0 if t.is_floating_point() else 255.0)
    hsv = _rgb2hsv(f)
    hsv[0] = torch.fmod(hsv[0] + hue_factor + 1.0, 1.0)
    out = _hsv2rgb(hsv)
    if not t.is_floating_point():
        out = (out * 255.0).round().to(t.dtype)
    return back(out)


def _affine_grid(h, w, matrix, device, out_hw=None):
    """Inverse affine matrix (output → input pixel coords, paddle/PIL convention) → sampling grid."""
    oh, ow = out_hw or (h, w)
    a, b, c, d, e, f = matrix
    ys, xs = torch.meshgrid(torch.arange(oh, device=device, dtype=torch.float32) + 0.5,
                            torch.arange(ow, device=device, dtype=torch.float32) + 0.5, indexing='ij')
    sx = a * xs + b * ys + c
    sy = d * xs + e * ys + f
    gx = sx / w * 2 - 1
    gy = sy / h * 2 - 1
    return torch.stack([gx, gy], -1).unsqueeze(0)


def _get_inverse_affine_matrix(center, angle, translate, scale, shear):
    rot = math.radians(angle)
    sx, sy = [math.radians(s) for s in shear]
    cx, cy = center
    tx, ty = translate
    a = math.cos(rot - sy) / math.cos(sy)
    b = -math.cos(rot - sy) * math.tan(sx) / math.cos(sy) - math.sin(rot)
    c = math.sin(rot - sy) / math.cos(sy)
    d = -math.sin(rot - sy) * math.tan(sx) / math.cos(sy) + math.cos(rot)
    m = [d, -b, 0.0, -c, a, 0.0]
    m = [x / scale for x in m]
    m[2] += m[0] * (-cx - tx) + m[1] * (-cy - ty)
    m[5] += m[3] * (-cx - tx) + m[4] * (-cy - ty)
    m[2] += cx
    m[5] += cy
    return m


def _warp(t, grid, interpolation, fill):
    x = t.unsqueeze(0).float()
    mode = 'nearest' if interpolation == 'nearest' else 'bilinear'
    if fill is not None and fill != 0:
        ones = torch.ones_like(x[:, :1])
        x = torch.cat([x, ones], 1)
        out = TF.grid_sample(x, grid, mode=mode, padding_mode='zeros', align_corners=False)
        mask = out[:, -1:]
        out = out[:, :-1]
        fillv = torch.tensor(fill if isinstance(fill, (list, tuple)) else [fill] * out.shape[1],
                             dtype=out.dtype, device=out.device).view(1, -1, 1, 1)
        out = out * mask + fillv * (1 - mask)
    else:
        out = TF.grid_sample(x, grid, mode=mode, padding_mode='zeros', align_corners=False)
    out = out[0]
    if not t.is_floating_point():
        out = out.round().clamp(0, 255).to(t.dtype)
    return out


def affine(img, angle, translate, scale, shear, interpolation='nearest', fill=0, center=None):
    t, back = _in(img)
    h, w = _size_hw(t)
    if isinstance(shear, numbers.Number):
        shear = [shear, 0.0]
    c = center if center is not None else (w * 0.5, h * 0.5)
    m = _get_inverse_affine_matrix(c, -angle, translate, scale, shear)
    return back(_warp(t, _affine_grid(h, w, m, t.device), interpolation, fill))


def rotate(img, angle, interpolation='nearest', expand=False, center=None, fill=0):
    t, back = _in(img)
    h, w = _size_hw(t)
    c = center if center is not None else (w * 0.5, h * 0.5)
    m = _get_inverse_affine_matrix(c, -angle, (0, 0), 1.0, (0.0, 0.0))
    out_hw = None
    if expand:
        corners = [(0, 0), (w, 0), (w, h), (0, h)]
        rot = math.radians(angle)
        xs = [(x - c[0]) * math.cos(rot) + (y - c[1]) * math.sin(rot) for x, y in corners]
        ys = [-(x - c[0]) * math.sin(rot) + (y - c[1]) * math.cos(rot) for x, y in corners]
        ow, oh = int(math.ceil(max(xs) - min(xs))), int(math.ceil(max(ys) - min(ys)))
        m[2] += m[0] * ((w - ow) / 2) + m[1] * ((h - oh) / 2)
        m[5] += m[3] * ((w - ow) / 2) + m[4] * ((h - oh) / 2)
        out_hw = (oh, ow)
    return back(_warp(t, _affine_grid(h, w, m, t.device, out_hw), interpolation, fill))


def _get_perspective_coeffs(startpoints, endpoints):
    a = np.zeros((8, 8))
    b = np.zeros(8)
    for i, (p1, p2) in enumerate(zip(endpoints, startpoints)):
        a[2 * i] = [p1[0], p1[1], 1, 0, 0, 0, -p2[0] * p1[0], -p2[0] * p1[1]]
        a[2 * i + 1] = [0, 0, 0, p1[0], p1[1], 1, -p2[1] * p1[0], -p2[1] * p1[1]]
        b[2 * i], b[2 * i + 1] = p2
    return np.linalg.lstsq(a, b, rcond=None)[0].tolist()


def perspective(img, startpoints, endpoints, interpolation='nearest', fill=0):
    t, back = _in(img)
    h, w = _size_hw(t)
    a, b, c, d, e, f, g, hh = _get_perspective_coeffs(startpoints, endpoints)
    ys, xs = torch.meshgrid(torch.arange(h, dtype=torch.float32, device=t.device) + 0.5,
                            torch.arange(w, dtype=torch.float32, device=t.device) + 0.5, indexing='ij')
    den = g * xs + hh * ys + 1
    sx = (a * xs + b * ys + c) / den
    sy = (d * xs + e * ys + f) / den
    grid = torch.stack([sx / w * 2 - 1, sy / h * 2 - 1], -1).unsqueeze(0)
    return back(_warp(t, grid, interpolation, fill))


def to_grayscale(img, num_output_channels=1):
    t, back = _in(img)
    g = _gray(t)
    if num_output_channels == 3:
        g = g.expand(3, -1, -1)
    if not t.is_floating_point():
        g = g.round().to(t.dtype)
    if _is_pil_image(img):
        arr = g[0].numpy() if num_output_channels == 1 else g.permute(1, 2, 0).numpy()
        return Image.fromarray(arr.astype(np.uint8), 'L' if num_output_channels == 1 else 'RGB')
    return back(g)


def normalize(img, mean, std, data_format='CHW', to_rgb=False):
    if _is_pil_image(img):
        img = np.array(img).astype(np.float32)
        data_format = 'HWC'
    if isinstance(img, np.ndarray):
        m, s = np.asarray(mean, np.float32), np.asarray(std, np.float32)
        if data_format.upper() == 'CHW':
            m, s = m.reshape(-1, 1, 1), s.reshape(-1, 1, 1)
            if to_rgb:
                img = img[::-1]
        elif to_rgb:
            img = img[..., ::-1]
        return (img.astype(np.float32) - m) / s
    t = _unwrap(img).float()
    m = torch.as_tensor(mean, dtype=t.dtype, device=t.device)
    s = torch.as_tensor(std, dtype=t.dtype, device=t.device)
    if data_format.upper() == 'CHW':
        m, s = m.view(-1, 1, 1), s.view(-1, 1, 1)
        if to_rgb:
            t = t.flip(0)
    elif to_rgb:
        t = t.flip(-1)
    return _wrap((t - m) / s)


def erase(img, i, j, h, w, v, inplace=False):
    t, back = _in(img)
    out = t if inplace else t.clone()
    vv = _unwrap(v) if isinstance(v, Tensor) else torch.as_tensor(v, dtype=out.dtype)
    out[:, i:i + h, j:j + w] = vv.to(out.dtype)
    return back(out)
