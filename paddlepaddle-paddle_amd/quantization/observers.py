"""paddle.quantization.observers (reference: quantization/observers/__init__.py)."""
from . import AbsmaxObserver, AbsmaxObserverLayer, GroupWiseWeightObserver, GroupWiseWeightObserverLayer  # noqa: F401
