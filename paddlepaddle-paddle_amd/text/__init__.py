"""paddle.text (reference: python/paddle/text/viterbi_decode.py, text/datasets/*).

``viterbi_decode`` runs the whole batch on the device: one [B, T, T] max-plus step per time
step, length-masked, then a backpointer walk.  Dataset classes need downloads in the
reference; here they read local files only (``data_file=``) — there is no network.
"""
import torch

from ..core.tensor import _wrap, _unwrap
from ..nn.layer.layers import Layer
from ..io import Dataset


def viterbi_decode(potentials, transition_params, lengths, include_bos_eos_tag=True, name=None):
    pot, trans, lens = _unwrap(potentials), _unwrap(transition_params), _unwrap(lengths).long()
    B, L, T = pot.shape
    alpha = pot[:, 0]
    if include_bos_eos_tag:
        alpha = alpha + trans[-1].unsqueeze(0)          # from the start tag (last row)
    ident = torch.arange(T, device=pot.device).expand(B, T)
    bps = []
    for t in range(1, L):
        s = alpha.unsqueeze(2) + trans.unsqueeze(0)      # [B, from, to]
        best, idx = s.max(1)
        new = best + pot[:, t]
        live = (t < lens).unsqueeze(1)
        alpha = torch.where(live, new, alpha)
        bps.append(torch.where(live, idx, ident))
    if include_bos_eos_tag:
        alpha = alpha + trans[:, -2].unsqueeze(0)        # into the stop tag (second-to-last column)
    score, last = alpha.max(-1)
    path = [last]
    for bp in reversed(bps):
        last = bp.gather(1, last.unsqueeze(1)).squeeze(1)
        path.append(last)
    paths = torch.stack(path[::-1], 1)
    maxlen = int(lens.max().item()) if lens.numel() else 0
    paths = paths[:, :maxlen]
    paths = paths.masked_fill(torch.arange(maxlen, device=pot.device).unsqueeze(0) >= lens.unsqueeze(1), 0)
    return _wrap(score), _wrap(paths)


class ViterbiDecoder(Layer):
    def __init__(self, transitions, include_bos_eos_tag=True, name=None):
        super().__init__()
        self.transitions = transitions
        self.include_bos_eos_tag = include_bos_eos_tag

    def forward(self, potentials, lengths):
        return viterbi_decode(potentials, self.transitions, lengths, self.include_bos_eos_tag)


from . import datasets  # noqa: E402,F401
from .datasets import Conll05st, Imdb, Imikolov, Movielens, UCIHousing, WMT14, WMT16  # noqa: E402,F401

__all__ = ['Conll05st', 'Imdb', 'Imikolov', 'Movielens', 'UCIHousing', 'WMT14', 'WMT16', 'ViterbiDecoder',
           'viterbi_decode']
