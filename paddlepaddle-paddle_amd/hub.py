"""paddle.hub (reference: python/paddle/hub.py): hubconf-based model listing / help / loading
from a local directory (no network here)."""
from .hapi.hub import help, list, load  # noqa: F401,A004

__all__ = ['list', 'help', 'load']
