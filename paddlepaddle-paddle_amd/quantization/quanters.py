"""paddle.quantization.quanters (reference: quantization/quanters/__init__.py)."""
from . import FakeQuanterWithAbsMaxObserver, FakeQuanterWithAbsMaxObserverLayer  # noqa: F401
