"""paddle.quantization.observers (reference: quantization/observers/__init__.py)."""
from . import AbsmaxObserver, AbsmaxObserverLayer  # noqa: F401
