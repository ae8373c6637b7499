"""paddle.set_printoptions (reference: python/paddle/tensor/to_string.py set_printoptions)."""
import numpy as np


_opts = {'precision': 8}


def set_printoptions(precision=None, threshold=None, edgeitems=None, sci_mode=None, linewidth=None):
    kw = {}
    if precision is not None:
        kw['precision'] = precision
        _opts['precision'] = precision
    if threshold is not None:
        kw['threshold'] = threshold
    if edgeitems is not None:
        kw['edgeitems'] = edgeitems
    if linewidth is not None:
        kw['linewidth'] = linewidth
    if sci_mode is not None:
        kw['suppress'] = not sci_mode
    np.set_printoptions(**kw)
