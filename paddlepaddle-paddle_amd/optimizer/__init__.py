"""paddle.optimizer (reference: python/paddle/optimizer/__init__.py)."""
from .optimizer import Optimizer  # noqa: F401
from .algorithms import (SGD, Momentum, Adam, AdamW, Adamax, Adagrad, Adadelta, RMSProp, Lamb, NAdam, RAdam,  # noqa: F401
                         ASGD, Rprop, LBFGS)
from . import lr  # noqa: F401
