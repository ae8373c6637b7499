"""paddle.decomposition (reference: python/paddle/decomposition/__init__.py): composite-op ->
primitive-op decomposition of static programs (``decompose``) with a rule registry
(``register.register_decomp``)."""
from . import rules  # noqa: F401
from .decomp import decompose  # noqa: F401
from .register import register_decomp, get_decomp_rule  # noqa: F401
