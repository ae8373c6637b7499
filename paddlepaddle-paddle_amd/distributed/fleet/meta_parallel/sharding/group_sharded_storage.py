"""group_sharded_storage (reference: meta_parallel/sharding/group_sharded_storage.py): contiguous
parameter / gradient storages.  The engine's equivalent is parallel.flat_buffer.FlatBuffer (one
flat data + grad buffer per unit, parameters as views into it); these classes expose the reference
names over it."""
import torch

from .....parallel.flat_buffer import FlatBuffer


class InternalStorage:
    def __init__(self, size, dtype, device, convert_cpu=False):
        dev = 'cpu' if convert_cpu or device == 'cpu' else ('cuda' if torch.cuda.is_available() else 'cpu')
        self.buffer = torch.zeros(int(size), dtype=dtype, device=dev)
        self._params = []
        self._fill = 0

    def to(self, device, dtype=None, keep_alignment=True):
        self.buffer = self.buffer.to(device=device, dtype=dtype or self.buffer.dtype)
        return self


class ParamStorage(InternalStorage):
    """Parameters packed into one buffer (``add_rank_params``): each becomes a view of it."""

    def __init__(self, size, dtype, device):
        super().__init__(size, dtype, device)
        self.param2align = {}

    def add_rank_params(self, trainable_params, param2align, convert_gpu=True):
        self._fb = FlatBuffer(list(trainable_params))
        self.buffer = self._fb.data
        self._params = list(trainable_params)
        self.param2align = dict(param2align or {})


class GradStorage(InternalStorage):
    """Gradient buffer of a parameter group (the engine keeps gradients in the unit's flat grad)."""

    def __init__(self, size, dtype, device, destination, parm2align, convert_cpu=False):
        super().__init__(size, dtype, device, convert_cpu)
        self.destination = destination
        self._param2align = parm2align
        self.params_checked_in = 0
        self.sent = False

    def reset_checked_in(self):
        self.params_checked_in = 0
        self.sent = False

    @property
    def all_checked_in(self):
        return len(self._params) == self.params_checked_in

    def can_add_grad_view(self, param, align):
        return self._fill + param._t.numel() + align <= self.buffer.numel()

    def add_grad(self, param, align):
        n = param._t.numel()
        view = self.buffer[self._fill:self._fill + n].view(param._t.shape)
        self._params.append(param)
        self._fill += n + align
        return view
