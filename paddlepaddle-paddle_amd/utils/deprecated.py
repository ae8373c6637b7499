"""paddle.utils.deprecated decorator (reference: python/paddle/utils/deprecated.py)."""
import functools
import warnings


def deprecated(update_to="", since="", reason="", level=0):
    def deco(fn):
        msg = f"API {fn.__module__}.{fn.__name__} is deprecated" + (f" since {since}" if since else "") + \
            (f", use {update_to} instead" if update_to else "") + (f". Reason: {reason}" if reason else "")

        @functools.wraps(fn)
        def wrapper(*a, **k):
            if level == 2:
                raise RuntimeError(msg)
            if level == 1 or level == 0:
                warnings.warn(msg, DeprecationWarning, stacklevel=2)
            return fn(*a, **k)
        return wrapper
    return deco
