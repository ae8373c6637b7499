"""paddle.hapi (reference: python/paddle/hapi/__init__.py)."""
from .model import Model  # noqa: F401
from .model_summary import summary  # noqa: F401
from .dynamic_flops import flops  # noqa: F401
from . import callbacks  # noqa: F401
from . import hub  # noqa: F401
