"""paddle.utils.dlpack (reference: python/paddle/utils/dlpack.py): zero-copy exchange with any
DLPack producer/consumer (HIP device memory is exported as kDLROCM)."""
import torch

from ..core.tensor import Tensor, _wrap, _unwrap


def to_dlpack(x):
    return torch.utils.dlpack.to_dlpack(_unwrap(x) if isinstance(x, Tensor) else x)


def from_dlpack(dlpack):
    return _wrap(torch.utils.dlpack.from_dlpack(dlpack))
