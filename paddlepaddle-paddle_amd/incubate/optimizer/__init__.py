"""incubate optimizers (reference: python/paddle/incubate/optimizer/lookahead.py,
modelaverage.py)."""
import contextlib

import torch

from ...core.tensor import _unwrap


class LookAhead:
    """k fast steps of the inner optimizer, then slow ← slow + alpha (fast − slow), fast ← slow."""

    def __init__(self, inner_optimizer, alpha=0.5, k=5, name=None):
        self.inner_optimizer = inner_optimizer
        self.alpha, self.k = alpha, k
        self._step = 0
        self._slow = {}
        self._parameter_list = inner_optimizer._parameter_list

    @torch.no_grad()
    def step(self):
        self.inner_optimizer.step()
        self._step += 1
        if self._step % self.k == 0:
            for p in self._parameter_list:
                t = _unwrap(p)
                s = self._slow.get(id(p))
                if s is None:
                    s = self._slow[id(p)] = t.detach().clone()
                s.add_(t - s, alpha=self.alpha)
                t.copy_(s)
        elif self._step == 1:
            for p in self._parameter_list:
                self._slow.setdefault(id(p), _unwrap(p).detach().clone())

    def clear_grad(self, set_to_zero=True):
        self.inner_optimizer.clear_grad(set_to_zero)

    def minimize(self, loss, *a, **k):
        loss.backward()
        self.step()

    def __getattr__(self, n):
        return getattr(self.inner_optimizer, n)


class ModelAverage:
    """Running average of parameters over a window; ``apply()`` swaps averages in."""

    def __init__(self, average_window_rate, parameters=None, min_average_window=10000, max_average_window=10000,
                 name=None):
        self._params = list(parameters or [])
        self.rate, self.min_w, self.max_w = average_window_rate, min_average_window, max_average_window
        self._sum = {id(p): torch.zeros_like(_unwrap(p), dtype=torch.float32) for p in self._params}
        self._n = 0
        self._backup = {}

    @torch.no_grad()
    def step(self):
        self._n += 1
        window = max(self.min_w, min(self.max_w, int(self._n * self.rate) or 1))
        for p in self._params:
            s = self._sum[id(p)]
            if self._n > window:
                s.mul_((window - 1) / window)
            s.add_(_unwrap(p).float())

    def minimize(self, loss, *a, **k):
        self.step()

    @contextlib.contextmanager
    def apply(self, executor=None, need_restore=True):
        with torch.no_grad():
            cnt = max(1, min(self._n, max(self.min_w, min(self.max_w, int(self._n * self.rate) or 1))))
            for p in self._params:
                t = _unwrap(p)
                self._backup[id(p)] = t.detach().clone()
                t.copy_((self._sum[id(p)] / cnt).to(t.dtype))
        try:
            yield
        finally:
            if need_restore:
                self.restore()

    def restore(self, executor=None):
        with torch.no_grad():
            for p in self._params:
                if id(p) in self._backup:
                    _unwrap(p).copy_(self._backup.pop(id(p)))


from ...optimizer.algorithms import LBFGS  # noqa: E402,F401  (reference: incubate/optimizer/lbfgs.py)
from . import functional  # noqa: E402,F401

from .distributed_fused_lamb import DistributedFusedLamb  # noqa: E402,F401
