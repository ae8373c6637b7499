"""Reference auto_parallel/strategy.py: the auto-parallel Strategy (defined in api.py)."""
from .api import Strategy  # noqa: F401
