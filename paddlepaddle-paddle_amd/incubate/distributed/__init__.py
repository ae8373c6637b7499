"""paddle.incubate.distributed (reference: python/paddle/incubate/distributed/)."""
from . import models  # noqa: F401
from . import utils  # noqa: F401
from . import fleet  # noqa: F401
