"""paddle.incubate.distributed.utils (reference: python/paddle/incubate/distributed/utils/)."""
from . import io  # noqa: F401
