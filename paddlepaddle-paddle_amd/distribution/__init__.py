"""paddle.distribution (reference: python/paddle/distribution/*.py).

Each distribution keeps its parameters as paddle Tensors and evaluates densities, samples and
entropies with the device kernels behind ``torch.distributions`` (so parameters keep their
autograd graph for reparameterised sampling).  Paddle's API surface and its quirks are
preserved: ``sample(shape)`` is non-differentiable and ``rsample`` reparameterised,
``prob``/``probs`` = exp(log_prob), ``Categorical(logits)`` normalises ``logits`` by their sum
for ``probs`` but uses softmax for ``entropy``/``kl_divergence``/``sample`` (categorical.py:121,
:237, :180).
"""
import math

import torch
import torch.distributions as D

from ..core.tensor import Tensor, _wrap, _unwrap
from . import transform  # noqa: F401
from .transform import *  # noqa: F401,F403


def _t(x, like=None):
    if isinstance(x, Tensor):
        return x._t
    if isinstance(x, torch.Tensor):
        return x
    from ..core.place import current_device
    dt = like.dtype if isinstance(like, torch.Tensor) else torch.float32
    dev = like.device if isinstance(like, torch.Tensor) else current_device()
    return torch.as_tensor(x, dtype=dt if not isinstance(x, bool) else torch.bool, device=dev)


def _shape(s):
    if s is None:
        return torch.Size()
    if isinstance(s, int):
        return torch.Size([s])
    return torch.Size(list(s))


class Distribution:
    def __init__(self, batch_shape=(), event_shape=()):
        self._batch_shape = tuple(batch_shape)
        self._event_shape = tuple(event_shape)

    @property
    def batch_shape(self):
        return self._batch_shape

    @property
    def event_shape(self):
        return self._event_shape

    def sample(self, shape=()):
        raise NotImplementedError

    def rsample(self, shape=()):
        raise NotImplementedError

    def entropy(self):
        raise NotImplementedError

    def log_prob(self, value):
        raise NotImplementedError

    def prob(self, value):
        return _wrap(torch.exp(_unwrap(self.log_prob(value))))

    probs = prob

    def kl_divergence(self, other):
        return kl_divergence(self, other)

    def _extend_shape(self, sample_shape):
        return tuple(sample_shape) + self._batch_shape + self._event_shape


class _TorchBacked(Distribution):
    """Shared plumbing: ``self._d`` is the torch distribution over unwrapped parameters."""
    _has_rsample = True

    def _init(self, d):
        self._d = d
        Distribution.__init__(self, tuple(d.batch_shape), tuple(d.event_shape))

    @property
    def mean(self):
        return _wrap(self._d.mean)

    @property
    def variance(self):
        return _wrap(self._d.variance)

    @property
    def stddev(self):
        return _wrap(self._d.stddev)

    def sample(self, shape=(), seed=0):
        with torch.no_grad():
            return _wrap(self._d.sample(_shape(shape)))

    def rsample(self, shape=()):
        if not self._d.has_rsample:
            raise NotImplementedError(f"{type(self).__name__} has no reparameterised sampler")
        return _wrap(self._d.rsample(_shape(shape)))

    def log_prob(self, value):
        return _wrap(self._d.log_prob(_t(value, self._param_like())))

    def entropy(self):
        return _wrap(self._d.entropy())

    def cdf(self, value):
        return _wrap(self._d.cdf(_t(value, self._param_like())))

    def icdf(self, value):
        return _wrap(self._d.icdf(_t(value, self._param_like())))

    def _param_like(self):
        for v in vars(self._d).values():
            if isinstance(v, torch.Tensor) and v.is_floating_point():
                return v
        return None


class ExponentialFamily(_TorchBacked):
    pass


class Normal(ExponentialFamily):
    def __init__(self, loc, scale, name=None):
        self.loc, self.scale = _wrap(_t(loc)), None
        sc = _t(scale, self.loc._t)
        self.scale = _wrap(sc)
        self.name = name or 'Normal'
        self._init(D.Normal(self.loc._t, sc, validate_args=False))

    def probs(self, value):
        return self.prob(value)


class Uniform(_TorchBacked):
    def __init__(self, low, high, name=None):
        lo = _t(low)
        self.low, self.high = _wrap(lo), _wrap(_t(high, lo))
        self.name = name or 'Uniform'
        self._init(D.Uniform(self.low._t, self.high._t, validate_args=False))


class Bernoulli(ExponentialFamily):
    def __init__(self, probs, name=None):
        self.probs_ = _wrap(_t(probs))
        self.name = name or 'Bernoulli'
        self._init(D.Bernoulli(probs=self.probs_._t, validate_args=False))

    @property
    def probs(self):
        return self.probs_

    def rsample(self, shape=(), temperature=1.0):
        """Relaxed (Gumbel-sigmoid) sample: differentiable w.r.t. probs (bernoulli.py:193)."""
        p = self.probs_._t
        u = torch.rand(_shape(shape) + p.shape, device=p.device, dtype=p.dtype).clamp(1e-6, 1 - 1e-6)
        logits = torch.log(p) - torch.log1p(-p)
        return _wrap(torch.sigmoid((logits + torch.log(u) - torch.log1p(-u)) / temperature))

    def prob(self, value):
        return _wrap(torch.exp(self._d.log_prob(_t(value, self.probs_._t))))


class Beta(ExponentialFamily):
    def __init__(self, alpha, beta, name=None):
        a = _t(alpha)
        self.alpha, self.beta = _wrap(a), _wrap(_t(beta, a))
        self._init(D.Beta(self.alpha._t, self.beta._t, validate_args=False))


class Dirichlet(ExponentialFamily):
    def __init__(self, concentration, name=None):
        self.concentration = _wrap(_t(concentration))
        self._init(D.Dirichlet(self.concentration._t, validate_args=False))


class Exponential(ExponentialFamily):
    def __init__(self, rate, name=None):
        self.rate = _wrap(_t(rate))
        self._init(D.Exponential(self.rate._t, validate_args=False))


class Gamma(ExponentialFamily):
    def __init__(self, concentration, rate, name=None):
        c = _t(concentration)
        self.concentration, self.rate = _wrap(c), _wrap(_t(rate, c))
        self._init(D.Gamma(self.concentration._t, self.rate._t, validate_args=False))


class Laplace(_TorchBacked):
    def __init__(self, loc, scale, name=None):
        lo = _t(loc)
        self.loc, self.scale = _wrap(lo), _wrap(_t(scale, lo))
        self._init(D.Laplace(self.loc._t, self.scale._t, validate_args=False))


class LogNormal(_TorchBacked):
    def __init__(self, loc, scale, name=None):
        lo = _t(loc)
        self.loc, self.scale = _wrap(lo), _wrap(_t(scale, lo))
        self._init(D.LogNormal(self.loc._t, self.scale._t, validate_args=False))


class Gumbel(_TorchBacked):
    def __init__(self, loc, scale, name=None):
        lo = _t(loc)
        self.loc, self.scale = _wrap(lo), _wrap(_t(scale, lo))
        self._init(D.Gumbel(self.loc._t, self.scale._t, validate_args=False))

    def rsample(self, shape=()):
        lo, sc = self.loc._t, self.scale._t
        u = torch.rand(_shape(shape) + torch.broadcast_shapes(lo.shape, sc.shape), device=lo.device,
                       dtype=lo.dtype).clamp(1e-12, 1 - 1e-7)
        return _wrap(lo - sc * torch.log(-torch.log(u)))


class Cauchy(_TorchBacked):
    def __init__(self, loc, scale, name=None):
        lo = _t(loc)
        self.loc, self.scale = _wrap(lo), _wrap(_t(scale, lo))
        self._init(D.Cauchy(self.loc._t, self.scale._t, validate_args=False))


class Geometric(_TorchBacked):
    def __init__(self, probs):
        self.probs_ = _wrap(_t(probs))
        self._init(D.Geometric(probs=self.probs_._t, validate_args=False))

    @property
    def probs(self):
        return self.probs_

    def pmf(self, k):
        return self.prob(k)

    def log_pmf(self, k):
        return self.log_prob(k)


class Binomial(_TorchBacked):
    def __init__(self, total_count, probs):
        p = _t(probs)
        self.total_count, self.probs_ = _wrap(_t(total_count, p)), _wrap(p)
        self._init(D.Binomial(self.total_count._t, probs=p, validate_args=False))


class Poisson(ExponentialFamily):
    def __init__(self, rate):
        self.rate = _wrap(_t(rate))
        self._init(D.Poisson(self.rate._t, validate_args=False))


class StudentT(_TorchBacked):
    def __init__(self, df, loc, scale, name=None):
        d = _t(df)
        self.df, self.loc, self.scale = _wrap(d), _wrap(_t(loc, d)), _wrap(_t(scale, d))
        self._init(D.StudentT(self.df._t, self.loc._t, self.scale._t, validate_args=False))


class Multinomial(_TorchBacked):
    def __init__(self, total_count, probs):
        self.total_count = int(total_count)
        self.probs_ = _wrap(_t(probs))
        self._init(D.Multinomial(self.total_count, probs=self.probs_._t, validate_args=False))


class MultivariateNormal(_TorchBacked):
    def __init__(self, loc, covariance_matrix=None, precision_matrix=None, scale_tril=None):
        lo = _t(loc)
        kw = {}
        if covariance_matrix is not None:
            kw['covariance_matrix'] = _t(covariance_matrix, lo)
        if precision_matrix is not None:
            kw['precision_matrix'] = _t(precision_matrix, lo)
        if scale_tril is not None:
            kw['scale_tril'] = _t(scale_tril, lo)
        self.loc = _wrap(lo)
        self._init(D.MultivariateNormal(lo, validate_args=False, **kw))


class ContinuousBernoulli(_TorchBacked):
    def __init__(self, probs, lims=(0.499, 0.501)):
        self.probs_ = _wrap(_t(probs))
        self._init(D.ContinuousBernoulli(probs=self.probs_._t, lims=lims, validate_args=False))


class Categorical(Distribution):
    def __init__(self, logits, name=None):
        self.logits = _wrap(_t(logits))
        self.name = name or 'Categorical'
        lg = self.logits._t
        self._prob = lg / lg.sum(-1, keepdim=True)
        super().__init__(tuple(lg.shape[:-1]), ())

    def sample(self, shape=()):
        lg = self.logits._t
        d = D.Categorical(logits=lg, validate_args=False)
        with torch.no_grad():
            return _wrap(d.sample(_shape(shape)))

    def entropy(self):
        return _wrap(D.Categorical(logits=self.logits._t, validate_args=False).entropy())

    def kl_divergence(self, other):
        p = torch.log_softmax(self.logits._t, -1)
        q = torch.log_softmax(other.logits._t, -1)
        return _wrap((p.exp() * (p - q)).sum(-1, keepdim=True))

    def probs(self, value):
        v = _t(value).long()
        if self._prob.dim() == 1:
            return _wrap(self._prob[v.reshape(-1)].reshape(v.shape))
        if v.dim() == 1:
            v = v.reshape([1] * (self._prob.dim() - 1) + [-1]).expand(*self._prob.shape[:-1], v.shape[0])
        return _wrap(torch.take_along_dim(self._prob, v, -1))

    def log_prob(self, value):
        return _wrap(torch.log(_unwrap(self.probs(value))))


class Independent(Distribution):
    def __init__(self, base, reinterpreted_batch_rank):
        self._base = base
        self._rank = int(reinterpreted_batch_rank)
        bs = tuple(base.batch_shape)
        super().__init__(bs[:len(bs) - self._rank], bs[len(bs) - self._rank:] + tuple(base.event_shape))

    @property
    def mean(self):
        return self._base.mean

    @property
    def variance(self):
        return self._base.variance

    def sample(self, shape=()):
        return self._base.sample(shape)

    def rsample(self, shape=()):
        return self._base.rsample(shape)

    def _sum(self, t):
        return t.sum(list(range(-self._rank, 0))) if self._rank else t

    def log_prob(self, value):
        return _wrap(self._sum(_unwrap(self._base.log_prob(value))))

    def entropy(self):
        return _wrap(self._sum(_unwrap(self._base.entropy())))


class TransformedDistribution(Distribution):
    def __init__(self, base, transforms):
        self._base = base
        self._transforms = list(transforms)
        from .transform import ChainTransform
        self._chain = ChainTransform(self._transforms)
        shape = tuple(base.batch_shape) + tuple(base.event_shape)
        out_shape = self._chain.forward_shape(shape)
        super().__init__(tuple(base.batch_shape), tuple(out_shape[len(base.batch_shape):]))

    def sample(self, shape=()):
        return self._chain.forward(self._base.sample(shape))

    def rsample(self, shape=()):
        return self._chain.forward(self._base.rsample(shape))

    def log_prob(self, value):
        x = self._chain.inverse(value)
        lp = _unwrap(self._base.log_prob(x)) - _unwrap(self._chain.forward_log_det_jacobian(x))
        return _wrap(lp)


# ----------------------------------------------------------------- KL registry
_KL = {}


def register_kl(cls_p, cls_q):
    def deco(fn):
        _KL[(cls_p, cls_q)] = fn
        return fn
    return deco


def kl_divergence(p, q):
    for (a, b), fn in _KL.items():
        if isinstance(p, a) and isinstance(q, b):
            return fn(p, q)
    if isinstance(p, _TorchBacked) and isinstance(q, _TorchBacked):
        return _wrap(D.kl_divergence(p._d, q._d))
    if isinstance(p, Categorical) and isinstance(q, Categorical):
        return p.kl_divergence(q)
    raise NotImplementedError(f"no KL registered for {type(p).__name__} || {type(q).__name__}")


@register_kl(Normal, Normal)
def _kl_normal(p, q):
    var_ratio = (p.scale._t / q.scale._t) ** 2
    t1 = ((p.loc._t - q.loc._t) / q.scale._t) ** 2
    return _wrap(0.5 * (var_ratio + t1 - 1 - torch.log(var_ratio)))


_ = math
__all__ = ['Bernoulli', 'Beta', 'Categorical', 'Cauchy', 'ContinuousBernoulli', 'Dirichlet', 'Distribution',
           'Exponential', 'ExponentialFamily', 'Multinomial', 'MultivariateNormal', 'Normal', 'Uniform',
           'kl_divergence', 'register_kl', 'Independent', 'TransformedDistribution', 'Laplace', 'LogNormal', 'Gamma',
           'Gumbel', 'Geometric', 'Binomial', 'Poisson', 'StudentT'] + transform.__all__
