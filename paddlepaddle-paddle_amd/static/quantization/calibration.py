"""Activation-threshold calibration of static post-training quantisation (reference:
python/paddle/static/quantization/post_training_quantization.py algos 'KL' / 'hist' / 'mse' /
'avg' / 'abs_max' / 'min_max', cal_kl_threshold.py).  Statistics are gathered on the device per
observed tensor: running abs-max, per-batch abs-max (for 'avg') and a 2048-bin histogram of |x|
over [0, abs-max of the first pass] (for 'hist' / 'KL' / 'mse')."""
import math

import torch

BINS = 2048


class Observer:
    def __init__(self):
        self.absmax = 0.0
        self.batch_max = []
        self.hist = None
        self.hist_max = None
        self.min = math.inf
        self.max = -math.inf

    def observe_range(self, x):
        x = x.detach()
        if not x.is_floating_point() or x.numel() == 0:
            return
        m = float(x.abs().amax())
        self.absmax = max(self.absmax, m)
        self.batch_max.append(m)
        self.min = min(self.min, float(x.amin()))
        self.max = max(self.max, float(x.amax()))

    def observe_hist(self, x):
        x = x.detach()
        if not x.is_floating_point() or x.numel() == 0 or self.hist_max is None or self.hist_max <= 0:
            return
        h = torch.histc(x.float().abs().reshape(-1), bins=BINS, min=0.0, max=self.hist_max)
        self.hist = h.cpu().double() if self.hist is None else self.hist + h.cpu().double()


def _hist_threshold(hist, hmax, percent):
    c = torch.cumsum(hist, 0)
    tot = float(c[-1])
    if tot <= 0:
        return hmax
    idx = int(torch.searchsorted(c, torch.tensor(percent * tot, dtype=c.dtype)))
    return (min(idx, BINS - 1) + 0.5) * hmax / BINS


def _kl_threshold(hist, hmax, bits):
    """The clipping bin whose quantised (2^(bits-1) levels) distribution is closest in KL divergence
    to the clipped reference distribution (outliers folded into the last kept bin)."""
    levels = 2 ** (bits - 1)
    h = hist.double()
    best, best_i = math.inf, BINS - 1
    start = max(levels, 128)
    for i in range(start, BINS + 1, 8):
        ref = h[:i].clone()
        ref[i - 1] += h[i:].sum()
        if ref.sum() <= 0:
            continue
        # quantise the first i bins into `levels` groups, expand back over the non-empty bins
        grp = torch.div(torch.arange(i, dtype=torch.long) * levels, i, rounding_mode='floor')
        sums = torch.zeros(levels, dtype=torch.float64).index_add_(0, grp, h[:i])
        nz = (h[:i] > 0).double()
        cnt = torch.zeros(levels, dtype=torch.float64).index_add_(0, grp, nz)
        q = torch.where(nz > 0, sums[grp] / cnt[grp].clamp(min=1), torch.zeros_like(nz))
        p = ref / ref.sum()
        qs = q.sum()
        if qs <= 0:
            continue
        q = q / qs
        m = p > 0
        if bool((q[m] <= 0).any()):
            q = torch.where(m & (q <= 0), torch.full_like(q, 1e-12), q)
        kl = float((p[m] * torch.log(p[m] / q[m])).sum())
        if kl < best:
            best, best_i = kl, i
    return (best_i + 0.5) * hmax / BINS


def _mse_threshold(hist, hmax, bits):
    """Threshold minimising the expected squared quant-dequant error over the histogram."""
    qmax = 2 ** (bits - 1) - 1
    centers = (torch.arange(BINS, dtype=torch.float64) + 0.5) * hmax / BINS
    h = hist.double()
    best, best_t = math.inf, hmax
    for k in range(BINS // 32, BINS + 1, 16):
        t = k * hmax / BINS
        step = t / qmax
        clip = (centers - t).clamp(min=0) ** 2
        err = float((h * torch.where(centers > t, clip, torch.full_like(centers, step * step / 12.0))).sum())
        if err < best:
            best, best_t = err, t
    return best_t


def threshold(obs, algo, bits=8, hist_percent=0.99999):
    algo = algo.lower() if isinstance(algo, str) else 'kl'
    if obs.absmax <= 0:
        return 1e-8
    if algo in ('abs_max', 'abs_max_channel'):
        return obs.absmax
    if algo == 'min_max':
        return max(abs(obs.min), abs(obs.max))
    if algo == 'avg':
        return sum(obs.batch_max) / max(1, len(obs.batch_max))
    if obs.hist is None:
        return obs.absmax
    if algo == 'hist':
        return _hist_threshold(obs.hist, obs.hist_max, hist_percent)
    if algo in ('kl',):
        return _kl_threshold(obs.hist, obs.hist_max, bits)
    if algo in ('mse', 'emd'):
        return _mse_threshold(obs.hist, obs.hist_max, bits)
    raise ValueError(f"unknown calibration algo {algo}")


def needs_hist(algo):
    return str(algo).lower() in ('kl', 'hist', 'mse', 'emd')
