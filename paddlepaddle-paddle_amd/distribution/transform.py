"""Bijective transforms (reference: python/paddle/distribution/transform.py)."""
import enum

import torch

from ..core.tensor import _wrap, _unwrap


class Type(enum.Enum):
    BIJECTION = 'bijection'
    INJECTION = 'injection'
    SURJECTION = 'surjection'
    OTHER = 'other'


def _u(x):
    return _unwrap(x) if not isinstance(x, torch.Tensor) else x


class Transform:
    _type = Type.INJECTION

    def __call__(self, x):
        return self.forward(x)

    def forward(self, x):
        return _wrap(self._forward(_u(x)))

    def inverse(self, y):
        return _wrap(self._inverse(_u(y)))

    def forward_log_det_jacobian(self, x):
        return _wrap(self._fldj(_u(x)))

    def inverse_log_det_jacobian(self, y):
        y = _u(y)
        return _wrap(-self._fldj(self._inverse(y)))

    def forward_shape(self, shape):
        return tuple(shape)

    def inverse_shape(self, shape):
        return tuple(shape)

    def _forward(self, x):
        raise NotImplementedError

    def _inverse(self, y):
        raise NotImplementedError

    def _fldj(self, x):
        raise NotImplementedError


class AbsTransform(Transform):
    _type = Type.SURJECTION

    def _forward(self, x):
        return x.abs()

    def inverse(self, y):
        y = _u(y)
        return _wrap(-y), _wrap(y)

    def _fldj(self, x):
        return torch.zeros_like(x)


class AffineTransform(Transform):
    _type = Type.BIJECTION

    def __init__(self, loc, scale):
        self.loc, self.scale = _u(loc), _u(scale)

    def _forward(self, x):
        return self.loc + self.scale * x

    def _inverse(self, y):
        return (y - self.loc) / self.scale

    def _fldj(self, x):
        return torch.log(torch.abs(self.scale)).expand_as(x) if self.scale.dim() else \
            torch.log(torch.abs(self.scale)) * torch.ones_like(x)


class ExpTransform(Transform):
    _type = Type.BIJECTION

    def _forward(self, x):
        return x.exp()

    def _inverse(self, y):
        return y.log()

    def _fldj(self, x):
        return x


class PowerTransform(Transform):
    _type = Type.BIJECTION

    def __init__(self, power):
        self.power = _u(power)

    def _forward(self, x):
        return x.pow(self.power)

    def _inverse(self, y):
        return y.pow(1 / self.power)

    def _fldj(self, x):
        return torch.log(torch.abs(self.power * x.pow(self.power - 1)))


class SigmoidTransform(Transform):
    _type = Type.BIJECTION

    def _forward(self, x):
        return torch.sigmoid(x)

    def _inverse(self, y):
        return torch.log(y) - torch.log1p(-y)

    def _fldj(self, x):
        return -torch.nn.functional.softplus(-x) - torch.nn.functional.softplus(x)


class TanhTransform(Transform):
    _type = Type.BIJECTION

    def _forward(self, x):
        return torch.tanh(x)

    def _inverse(self, y):
        return torch.atanh(y)

    def _fldj(self, x):
        return 2.0 * (torch.log(torch.tensor(2.0, dtype=x.dtype, device=x.device)) - x -
                      torch.nn.functional.softplus(-2.0 * x))


class SoftmaxTransform(Transform):
    _type = Type.OTHER

    def _forward(self, x):
        return torch.softmax(x, -1)

    def _inverse(self, y):
        return torch.log(y)

    def forward_log_det_jacobian(self, x):
        raise NotImplementedError("SoftmaxTransform is not a bijection")


class StickBreakingTransform(Transform):
    _type = Type.BIJECTION

    def _forward(self, x):
        offset = x.shape[-1] + 1 - torch.ones(x.shape[-1], device=x.device, dtype=x.dtype).cumsum(-1)
        z = torch.sigmoid(x - offset.log())
        zc = (1 - z).cumprod(-1)
        return torch.nn.functional.pad(z, (0, 1), value=1) * torch.nn.functional.pad(zc, (1, 0), value=1)

    def _inverse(self, y):
        y_crop = y[..., :-1]
        offset = y.shape[-1] - torch.ones(y_crop.shape[-1], device=y.device, dtype=y.dtype).cumsum(-1)
        sf = 1 - y_crop.cumsum(-1)
        sf = torch.clamp(sf, min=torch.finfo(y.dtype).tiny)
        return y_crop.log() - sf.log() + offset.log()

    def _fldj(self, x):
        offset = x.shape[-1] + 1 - torch.ones(x.shape[-1], device=x.device, dtype=x.dtype).cumsum(-1)
        x = x - offset.log()
        y = self._forward(x + offset.log())
        return (-x + torch.nn.functional.logsigmoid(x) + y[..., :-1].log()).sum(-1)

    def forward_shape(self, shape):
        return tuple(shape[:-1]) + (shape[-1] + 1,)

    def inverse_shape(self, shape):
        return tuple(shape[:-1]) + (shape[-1] - 1,)


class ReshapeTransform(Transform):
    _type = Type.BIJECTION

    def __init__(self, in_event_shape, out_event_shape):
        self.in_event_shape, self.out_event_shape = tuple(in_event_shape), tuple(out_event_shape)

    def _forward(self, x):
        lead = x.shape[:x.dim() - len(self.in_event_shape)]
        return x.reshape(tuple(lead) + self.out_event_shape)

    def _inverse(self, y):
        lead = y.shape[:y.dim() - len(self.out_event_shape)]
        return y.reshape(tuple(lead) + self.in_event_shape)

    def _fldj(self, x):
        return torch.zeros(x.shape[:x.dim() - len(self.in_event_shape)], device=x.device, dtype=x.dtype)

    def forward_shape(self, shape):
        return tuple(shape[:len(shape) - len(self.in_event_shape)]) + self.out_event_shape

    def inverse_shape(self, shape):
        return tuple(shape[:len(shape) - len(self.out_event_shape)]) + self.in_event_shape


class IndependentTransform(Transform):
    def __init__(self, base, reinterpreted_batch_rank):
        self.base, self.rank = base, int(reinterpreted_batch_rank)
        self._type = base._type

    def _forward(self, x):
        return self.base._forward(x)

    def _inverse(self, y):
        return self.base._inverse(y)

    def _fldj(self, x):
        j = self.base._fldj(x)
        return j.sum(list(range(-self.rank, 0))) if self.rank else j

    def forward_shape(self, shape):
        return self.base.forward_shape(shape)


class ChainTransform(Transform):
    def __init__(self, transforms):
        self.transforms = list(transforms)

    def _forward(self, x):
        for t in self.transforms:
            x = t._forward(x)
        return x

    def _inverse(self, y):
        for t in reversed(self.transforms):
            y = t._inverse(y)
        return y

    def _fldj(self, x):
        total = 0.
        for t in self.transforms:
            total = total + t._fldj(x)
            x = t._forward(x)
        return total

    def forward_shape(self, shape):
        for t in self.transforms:
            shape = t.forward_shape(shape)
        return shape

    def inverse_shape(self, shape):
        for t in reversed(self.transforms):
            shape = t.inverse_shape(shape)
        return shape


class StackTransform(Transform):
    def __init__(self, transforms, axis=0):
        self.transforms, self.axis = list(transforms), axis

    def _split(self, x):
        return x.unbind(self.axis)

    def _forward(self, x):
        return torch.stack([t._forward(c) for t, c in zip(self.transforms, self._split(x))], self.axis)

    def _inverse(self, y):
        return torch.stack([t._inverse(c) for t, c in zip(self.transforms, self._split(y))], self.axis)

    def _fldj(self, x):
        return torch.stack([t._fldj(c) for t, c in zip(self.transforms, self._split(x))], self.axis)


__all__ = ['Transform', 'AbsTransform', 'AffineTransform', 'ChainTransform', 'ExpTransform', 'IndependentTransform',
           'PowerTransform', 'ReshapeTransform', 'SigmoidTransform', 'SoftmaxTransform', 'StackTransform',
           'StickBreakingTransform', 'TanhTransform']
