"""paddle.incubate.distributed (reference: python/paddle/incubate/distributed/)."""
from . import models  # noqa: F401
