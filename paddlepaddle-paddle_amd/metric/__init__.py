"""paddle.metric (reference: python/paddle/metric/metrics.py — Metric:34, Accuracy:183,
Precision:333, Recall:462, Auc:594, accuracy:763).

``compute`` runs on device tensors (top-k on the GPU), ``update`` accumulates host-side
counters from the small per-batch results, ``accumulate`` reports."""
import abc

import numpy as np
import torch

from ..core.tensor import Tensor, _wrap, _unwrap


def _np(x):
    if isinstance(x, Tensor):
        t = x._t.detach()
        return (t.float() if t.dtype == torch.bfloat16 else t).cpu().numpy()
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    return np.asarray(x)


class Metric(metaclass=abc.ABCMeta):
    def __init__(self):
        pass

    @abc.abstractmethod
    def reset(self):
        raise NotImplementedError

    @abc.abstractmethod
    def update(self, *args):
        raise NotImplementedError

    @abc.abstractmethod
    def accumulate(self):
        raise NotImplementedError

    @abc.abstractmethod
    def name(self):
        raise NotImplementedError

    def compute(self, *args):
        return args


class Accuracy(Metric):
    def __init__(self, topk=(1,), name=None, *args, **kwargs):
        super().__init__()
        self.topk = tuple(topk)
        self.maxk = max(self.topk)
        name = name or 'acc'
        self._name = [f'{name}_top{k}' for k in self.topk] if self.maxk != 1 else [name]
        self.reset()

    def compute(self, pred, label, *args):
        p, l_ = _unwrap(pred), _unwrap(label)
        top = p.topk(self.maxk, dim=-1).indices
        if l_.dim() == 1 or (l_.dim() == 2 and l_.shape[-1] == 1):
            l_ = l_.reshape(-1, 1)
        elif l_.shape[-1] != 1:
            l_ = l_.argmax(-1, keepdim=True)
        return _wrap((top == l_.to(top.dtype)).float())

    def update(self, correct, *args):
        c = _np(correct)
        n = int(np.prod(c.shape[:-1]))
        accs = []
        for i, k in enumerate(self.topk):
            nc = float(c[..., :k].sum())
            accs.append(nc / max(n, 1))
            self.total[i] += nc
            self.count[i] += n
        return accs[0] if len(self.topk) == 1 else accs

    def reset(self):
        self.total = [0.0] * len(self.topk)
        self.count = [0] * len(self.topk)

    def accumulate(self):
        res = [t / c if c > 0 else 0.0 for t, c in zip(self.total, self.count)]
        return res[0] if len(self.topk) == 1 else res

    def name(self):
        return self._name


class Precision(Metric):
    """Binary precision; predictions are probabilities thresholded at 0.5."""

    def __init__(self, name='precision', *args, **kwargs):
        super().__init__()
        self._name = name
        self.reset()

    def update(self, preds, labels):
        p = (_np(preds).reshape(-1) >= 0.5).astype(np.int64)
        l_ = _np(labels).reshape(-1).astype(np.int64)
        self.tp += int(((p == 1) & (l_ == 1)).sum())
        self.fp += int(((p == 1) & (l_ == 0)).sum())

    def reset(self):
        self.tp = 0
        self.fp = 0

    def accumulate(self):
        ap = self.tp + self.fp
        return float(self.tp) / ap if ap != 0 else 0.0

    def name(self):
        return self._name


class Recall(Metric):
    def __init__(self, name='recall', *args, **kwargs):
        super().__init__()
        self._name = name
        self.reset()

    def update(self, preds, labels):
        p = (_np(preds).reshape(-1) >= 0.5).astype(np.int64)
        l_ = _np(labels).reshape(-1).astype(np.int64)
        self.tp += int(((p == 1) & (l_ == 1)).sum())
        self.fn += int(((p == 0) & (l_ == 1)).sum())

    def reset(self):
        self.tp = 0
        self.fn = 0

    def accumulate(self):
        recall = self.tp + self.fn
        return float(self.tp) / recall if recall != 0 else 0.0

    def name(self):
        return self._name


class Auc(Metric):
    """ROC / PR area from per-threshold positive/negative histograms (``num_thresholds``
    buckets over [0, 1]); preds are [N, 2] class probabilities or [N] / [N, 1] positives."""

    def __init__(self, curve='ROC', num_thresholds=4095, name='auc', *args, **kwargs):
        super().__init__()
        self._curve = curve
        self._num_thresholds = num_thresholds
        self._name = name
        self.reset()

    def update(self, preds, labels):
        p = _np(preds)
        if p.ndim == 2 and p.shape[1] == 2:
            p = p[:, 1]
        p = p.reshape(-1)
        l_ = _np(labels).reshape(-1)
        idx = np.clip((p * self._num_thresholds).astype(np.int64), 0, self._num_thresholds)
        np.add.at(self._stat_pos, idx[l_ == 1], 1)
        np.add.at(self._stat_neg, idx[l_ != 1], 1)

    @staticmethod
    def trapezoid_area(x1, x2, y1, y2):
        return abs(x1 - x2) * (y1 + y2) / 2.0

    def accumulate(self):
        tot_pos = tot_neg = 0.0
        auc = 0.0
        if self._curve == 'PR':
            tp = fp = 0.0
            prev_r, prev_p = 0.0, 1.0
            P = float(self._stat_pos.sum())
            if P == 0:
                return 0.0
            for i in range(self._num_thresholds, -1, -1):
                tp += self._stat_pos[i]
                fp += self._stat_neg[i]
                if tp + fp == 0:
                    continue
                r, pr = tp / P, tp / (tp + fp)
                auc += self.trapezoid_area(r, prev_r, pr, prev_p)
                prev_r, prev_p = r, pr
            return auc
        for i in range(self._num_thresholds, -1, -1):
            np_, nn_ = tot_pos, tot_neg
            tot_pos += self._stat_pos[i]
            tot_neg += self._stat_neg[i]
            auc += self.trapezoid_area(tot_neg, nn_, tot_pos, np_)
        return auc / tot_pos / tot_neg if tot_pos > 0.0 and tot_neg > 0.0 else 0.0

    def reset(self):
        self._stat_pos = np.zeros(self._num_thresholds + 1, dtype=np.int64)
        self._stat_neg = np.zeros(self._num_thresholds + 1, dtype=np.int64)

    def name(self):
        return self._name


def accuracy(input, label, k=1, correct=None, total=None, name=None):  # noqa: A002
    """Top-k accuracy of a batch as a 0-d float32 tensor (computed on device)."""
    p, l_ = _unwrap(input), _unwrap(label)
    top = p.topk(k, dim=-1).indices
    l_ = l_.reshape(-1, 1).to(top.dtype)
    hit = (top == l_).any(-1).float()
    if correct is not None:
        _unwrap(correct).copy_(hit.sum().to(_unwrap(correct).dtype))
    if total is not None:
        _unwrap(total).fill_(hit.numel())
    return _wrap(hit.mean())


__all__ = ['Metric', 'Accuracy', 'Precision', 'Recall', 'Auc', 'accuracy']
