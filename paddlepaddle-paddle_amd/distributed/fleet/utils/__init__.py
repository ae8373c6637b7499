"""paddle.distributed.fleet.utils (reference: python/paddle/distributed/fleet/utils/__init__.py)."""
from ..recompute import recompute  # noqa: F401
from . import sequence_parallel_utils  # noqa: F401
from .hybrid_parallel_util import fused_allreduce_gradients, broadcast_mp_parameters, broadcast_dp_parameters  # noqa: F401


class LocalFS:
    """Minimal local filesystem helper (reference fleet.utils.LocalFS)."""

    def mkdirs(self, p):
        import os
        os.makedirs(p, exist_ok=True)

    def is_exist(self, p):
        import os
        return os.path.exists(p)

    def ls_dir(self, p):
        import os
        ents = os.listdir(p)
        return [e for e in ents if os.path.isdir(os.path.join(p, e))], \
               [e for e in ents if os.path.isfile(os.path.join(p, e))]

    def delete(self, p):
        import shutil
        import os
        shutil.rmtree(p) if os.path.isdir(p) else (os.remove(p) if os.path.exists(p) else None)
