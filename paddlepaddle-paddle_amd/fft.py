"""paddle.fft (reference: python/paddle/fft.py).  Transforms run on rocFFT through torch.fft;
paddle's argument conventions (``axis``/``axes``, ``norm`` in {backward, ortho, forward})."""
import torch

from .core.tensor import _wrap, _unwrap

_NORMS = ('backward', 'ortho', 'forward')


def _norm(norm):
    if norm not in _NORMS:
        raise ValueError(f"Unexpected norm: {norm}. Norm should be forward, backward or ortho")
    return norm


def _axes(axes, x, n):
    if axes is None:
        return None if n is None else list(range(-len(n), 0))
    return list(axes)


def fft(x, n=None, axis=-1, norm="backward", name=None):
    return _wrap(torch.fft.fft(_unwrap(x), n, axis, _norm(norm)))


def ifft(x, n=None, axis=-1, norm="backward", name=None):
    return _wrap(torch.fft.ifft(_unwrap(x), n, axis, _norm(norm)))


def rfft(x, n=None, axis=-1, norm="backward", name=None):
    return _wrap(torch.fft.rfft(_unwrap(x), n, axis, _norm(norm)))


def irfft(x, n=None, axis=-1, norm="backward", name=None):
    return _wrap(torch.fft.irfft(_unwrap(x), n, axis, _norm(norm)))


def hfft(x, n=None, axis=-1, norm="backward", name=None):
    return _wrap(torch.fft.hfft(_unwrap(x), n, axis, _norm(norm)))


def ihfft(x, n=None, axis=-1, norm="backward", name=None):
    return _wrap(torch.fft.ihfft(_unwrap(x), n, axis, _norm(norm)))


def fftn(x, s=None, axes=None, norm="backward", name=None):
    return _wrap(torch.fft.fftn(_unwrap(x), s, _axes(axes, x, s), _norm(norm)))


def ifftn(x, s=None, axes=None, norm="backward", name=None):
    return _wrap(torch.fft.ifftn(_unwrap(x), s, _axes(axes, x, s), _norm(norm)))


def rfftn(x, s=None, axes=None, norm="backward", name=None):
    return _wrap(torch.fft.rfftn(_unwrap(x), s, _axes(axes, x, s), _norm(norm)))


def irfftn(x, s=None, axes=None, norm="backward", name=None):
    return _wrap(torch.fft.irfftn(_unwrap(x), s, _axes(axes, x, s), _norm(norm)))


def hfftn(x, s=None, axes=None, norm="backward", name=None):
    return _wrap(torch.fft.hfftn(_unwrap(x), s, _axes(axes, x, s), _norm(norm)))


def ihfftn(x, s=None, axes=None, norm="backward", name=None):
    return _wrap(torch.fft.ihfftn(_unwrap(x), s, _axes(axes, x, s), _norm(norm)))


def fft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    return fftn(x, s, axes, norm)


def ifft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    return ifftn(x, s, axes, norm)


def rfft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    return rfftn(x, s, axes, norm)


def irfft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    return irfftn(x, s, axes, norm)


def hfft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    return hfftn(x, s, axes, norm)


def ihfft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    return ihfftn(x, s, axes, norm)


def _dt(dtype):
    from .core.dtype import to_torch_dtype
    return to_torch_dtype(dtype) if dtype is not None else torch.get_default_dtype()


def fftfreq(n, d=1.0, dtype=None, name=None):
    from .core.place import current_device
    return _wrap(torch.fft.fftfreq(n, d, dtype=_dt(dtype), device=current_device()))


def rfftfreq(n, d=1.0, dtype=None, name=None):
    from .core.place import current_device
    return _wrap(torch.fft.rfftfreq(n, d, dtype=_dt(dtype), device=current_device()))


def fftshift(x, axes=None, name=None):
    return _wrap(torch.fft.fftshift(_unwrap(x), axes))


def ifftshift(x, axes=None, name=None):
    return _wrap(torch.fft.ifftshift(_unwrap(x), axes))


__all__ = ['fft', 'ifft', 'rfft', 'irfft', 'hfft', 'ihfft', 'fft2', 'ifft2', 'rfft2', 'irfft2', 'hfft2', 'ihfft2',
           'fftn', 'ifftn', 'rfftn', 'irfftn', 'hfftn', 'ihfftn', 'fftfreq', 'rfftfreq', 'fftshift', 'ifftshift']
