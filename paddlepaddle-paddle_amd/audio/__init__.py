"""paddle.audio (reference: python/paddle/audio/__init__.py)."""
from . import functional, features, backends  # noqa: F401
from .backends import load, info, save  # noqa: F401


class datasets:  # noqa: N801 - namespace mirror; ESC50/TESS need downloads
    class ESC50:
        def __init__(self, *a, **k):
            raise RuntimeError("ESC50 requires a download (no network access here)")

    class TESS(ESC50):
        pass


__all__ = ["functional", "features", "datasets", "backends", "load", "info", "save"]
