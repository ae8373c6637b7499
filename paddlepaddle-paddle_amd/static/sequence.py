"""LoD (level-1 variable-length sequence) tensors and the ``paddle.static.nn.sequence_*`` ops.

Reference: paddle/fluid/framework/lod_tensor.h (LoD = offsets of each sequence in the packed
rows), python/paddle/static/nn/sequence_lod.py (sequence_conv / softmax / pool / first_step /
last_step / slice / expand / expand_as / pad / unpad / reshape / scatter / enumerate) and the
phi kernels under paddle/phi/kernels/*sequence*.

Design: a LoD tensor is an ordinary Tensor whose rows pack the sequences back to back, plus a
``_lod`` attribute holding the level-1 offsets ([0, l0, l0+l1, ...]).  ``Tensor.set_lod`` /
``lod`` / ``set_recursive_sequence_lengths`` / ``recursive_sequence_lengths`` mirror the
reference LoDTensor API; ``create_lod_tensor`` builds one.  The ops read the offsets on the host
(they are per-batch metadata, as in the reference) and run vectorised torch work per batch: one
segment-id vector drives ``index_add``/``scatter_reduce`` instead of a Python loop per row.
Inside a static Program the ops are recorded as py-nodes; the Executor carries a fed tensor's LoD
through those nodes (static/executor.py), so a Program fed LoD tensors replays them.
"""
import numpy as np
import torch

from ..core.tensor import Tensor, _wrap, _unwrap


# ----------------------------------------------------------------------------- LoD plumbing
def get_lod(x):
    lod = x.__dict__.get('_lod') if isinstance(x, Tensor) else None
    if lod is None:
        raise ValueError("sequence op needs a LoD tensor (set_lod / create_lod_tensor / a fed LoD tensor)")
    return [int(v) for v in lod]


def with_lod(t, lod):
    out = t if isinstance(t, Tensor) else _wrap(t)
    out.__dict__['_lod'] = [int(v) for v in lod]
    return out


def lengths_to_offsets(lengths):
    return [0] + np.cumsum([int(l) for l in lengths]).tolist()


def offsets_to_lengths(lod):
    return [lod[i + 1] - lod[i] for i in range(len(lod) - 1)]


def _seg_ids(lod, device):
    lens = torch.tensor(offsets_to_lengths(lod), device=device)
    return torch.repeat_interleave(torch.arange(len(lens), device=device), lens)


def create_lod_tensor(data, recursive_seq_lens, place=None):
    """Reference: python/paddle/base/lod_tensor.py create_lod_tensor (level-1 lengths)."""
    from ..core.tensor import to_tensor
    if isinstance(data, list):
        data = np.concatenate([np.asarray(d).reshape(len(d), -1) for d in data], 0)
    t = data if isinstance(data, Tensor) else to_tensor(np.asarray(data))
    lens = recursive_seq_lens[-1] if recursive_seq_lens and isinstance(recursive_seq_lens[0], (list, tuple)) \
        else recursive_seq_lens
    lod = lengths_to_offsets(lens)
    if lod[-1] != t.shape[0]:
        raise ValueError(f"sum of sequence lengths {lod[-1]} != rows {t.shape[0]}")
    return with_lod(t, lod)


def install_tensor_methods():
    def set_lod(self, lod):
        lv = lod[-1] if lod and isinstance(lod[0], (list, tuple)) else lod
        self.__dict__['_lod'] = [int(v) for v in lv]

    def lod(self):
        l = self.__dict__.get('_lod')
        return [] if l is None else [list(l)]

    def set_recursive_sequence_lengths(self, lens):
        lv = lens[-1] if lens and isinstance(lens[0], (list, tuple)) else lens
        self.__dict__['_lod'] = lengths_to_offsets(lv)

    def recursive_sequence_lengths(self):
        l = self.__dict__.get('_lod')
        return [] if l is None else [offsets_to_lengths(l)]

    def has_valid_recursive_sequence_lengths(self):
        l = self.__dict__.get('_lod')
        return l is None or (l[0] == 0 and all(b >= a for a, b in zip(l, l[1:])) and l[-1] == self.shape[0])

    for f in (set_lod, lod, set_recursive_sequence_lengths, recursive_sequence_lengths,
              has_valid_recursive_sequence_lengths):
        setattr(Tensor, f.__name__, f)


# ----------------------------------------------------------------------------- ops
def sequence_pool(input, pool_type, is_test=False, pad_value=0.0):  # noqa: A002
    """Per-sequence reduction -> [num_seqs, D]: sum / average / sqrt / max / min / first / last."""
    lod = get_lod(input)
    x = _unwrap(input)
    x2 = x.reshape(x.shape[0], -1)
    n = len(lod) - 1
    lens = torch.tensor(offsets_to_lengths(lod), device=x.device)
    seg = _seg_ids(lod, x.device)
    pt = pool_type.lower()
    if pt in ('sum', 'average', 'sqrt'):
        out = torch.zeros(n, x2.shape[1], dtype=x2.dtype, device=x.device).index_add(0, seg, x2)
        if pt == 'average':
            out = out / lens.clamp_min(1).unsqueeze(1).to(out.dtype)
        elif pt == 'sqrt':
            out = out / lens.clamp_min(1).to(out.dtype).sqrt().unsqueeze(1)
    elif pt in ('max', 'min'):
        init = torch.full((n, x2.shape[1]), float('-inf') if pt == 'max' else float('inf'), dtype=x2.dtype,
                          device=x.device)
        out = init.scatter_reduce(0, seg.unsqueeze(1).expand_as(x2), x2, 'amax' if pt == 'max' else 'amin',
                                  include_self=True)
    elif pt in ('first', 'last'):
        starts = torch.tensor(lod[:-1], device=x.device)
        idx = starts if pt == 'first' else (starts + lens - 1).clamp_min(0)
        out = x2[idx.clamp(max=max(x2.shape[0] - 1, 0))]
    else:
        raise ValueError(f"unknown pool_type {pool_type}")
    out = torch.where((lens > 0).unsqueeze(1), out, torch.full_like(out, pad_value))
    return _wrap(out.reshape(n, *x.shape[1:]))


def sequence_first_step(input):  # noqa: A002
    return sequence_pool(input, 'first')


def sequence_last_step(input):  # noqa: A002
    return sequence_pool(input, 'last')


def sequence_softmax(input, use_cudnn=False, name=None):  # noqa: A002
    """Softmax over the time steps of each sequence (input [N] or [N, 1])."""
    lod = get_lod(input)
    x = _unwrap(input)
    v = x.reshape(-1)
    seg = _seg_ids(lod, x.device)
    n = len(lod) - 1
    mx = torch.full((n,), float('-inf'), dtype=v.dtype, device=x.device).scatter_reduce(0, seg, v, 'amax')
    e = torch.exp(v - mx[seg])
    s = torch.zeros(n, dtype=v.dtype, device=x.device).index_add(0, seg, e)
    return with_lod(_wrap((e / s[seg]).reshape(x.shape)), lod)


def _context_rows(x2, lod, filter_size, padding_start):
    """[N, filter_size * D] context projection: row t holds x[t + padding_start + j] for j in
    [0, filter_size), zero where that index leaves t's sequence (reference context_project.h)."""
    N, D = x2.shape
    seg = _seg_ids(lod, x2.device)
    starts = torch.tensor(lod[:-1], device=x2.device)[seg]
    ends = torch.tensor(lod[1:], device=x2.device)[seg]
    t = torch.arange(N, device=x2.device)
    cols = []
    for j in range(filter_size):
        src = t + padding_start + j
        ok = (src >= starts) & (src < ends)
        cols.append(torch.where(ok.unsqueeze(1), x2[src.clamp(0, max(N - 1, 0))], torch.zeros_like(x2)))
    return torch.cat(cols, 1)


def sequence_conv(input, num_filters, filter_size=3, filter_stride=1, padding=True, padding_start=None,  # noqa: A002
                  bias_attr=None, param_attr=None, act=None, name=None):
    from .. import nn as _nn
    from ..nn import functional as F
    lod = get_lod(input)
    x = _unwrap(input)
    D = x.shape[-1]
    if padding_start is None:
        padding_start = -int(filter_size // 2)
    lin = _nn.Linear(filter_size * D, num_filters, weight_attr=param_attr, bias_attr=bias_attr)
    ctx = _context_rows(x.reshape(x.shape[0], D), lod, filter_size, padding_start)
    out = lin(_wrap(ctx))
    if act is not None:
        out = getattr(F, act)(out)
    return with_lod(out, lod)


def sequence_slice(input, offset, length, name=None):  # noqa: A002
    lod = get_lod(input)
    x = _unwrap(input)
    off = np.asarray(_unwrap(offset).detach().cpu() if isinstance(offset, Tensor) else offset).reshape(-1)
    ln = np.asarray(_unwrap(length).detach().cpu() if isinstance(length, Tensor) else length).reshape(-1)
    idx, new = [], [0]
    for i in range(len(lod) - 1):
        s = lod[i] + int(off[i])
        if int(off[i]) + int(ln[i]) > lod[i + 1] - lod[i]:
            raise ValueError(f"sequence_slice: sequence {i} too short for offset {off[i]} + length {ln[i]}")
        idx.extend(range(s, s + int(ln[i])))
        new.append(new[-1] + int(ln[i]))
    return with_lod(_wrap(x[torch.tensor(idx, dtype=torch.long, device=x.device)]), new)


def sequence_expand(x, y, ref_level=-1, name=None):
    """Row (or sequence) i of x repeated len_i(y) times (reference sequence_expand_op)."""
    ylod = get_lod(y)
    t = _unwrap(x)
    reps = torch.tensor(offsets_to_lengths(ylod), device=t.device)
    xl = x.__dict__.get('_lod') if isinstance(x, Tensor) else None
    if xl is None:
        out = torch.repeat_interleave(t, reps, dim=0)
        return with_lod(_wrap(out), lengths_to_offsets([int(r) for r in reps.tolist()]))
    # x itself is a LoD tensor: its whole i-th sequence is repeated reps[i] times
    idx, new = [], [0]
    for i in range(len(xl) - 1):
        for _ in range(int(reps[i])):
            idx.extend(range(xl[i], xl[i + 1]))
            new.append(new[-1] + xl[i + 1] - xl[i])
    return with_lod(_wrap(t[torch.tensor(idx, dtype=torch.long, device=t.device)]), new)


def sequence_expand_as(x, y, name=None):
    ylod = get_lod(y)
    t = _unwrap(x)
    reps = torch.tensor(offsets_to_lengths(ylod), device=t.device)
    if t.shape[0] != len(reps):
        raise ValueError("sequence_expand_as: x must have one row per sequence of y")
    return with_lod(_wrap(torch.repeat_interleave(t, reps, dim=0)), ylod)


def sequence_pad(x, pad_value, maxlen=None, name=None):
    """-> (padded [num_seqs, maxlen, ...], lengths int64 [num_seqs])."""
    lod = get_lod(x)
    t = _unwrap(x)
    lens = offsets_to_lengths(lod)
    L = max(lens) if maxlen is None else int(maxlen)
    if lens and max(lens) > L:
        raise ValueError("sequence_pad: maxlen shorter than the longest sequence")
    pv = _unwrap(pad_value) if isinstance(pad_value, Tensor) else torch.tensor(pad_value)
    out = pv.to(t.dtype).to(t.device).expand(len(lens), L, *t.shape[1:]).clone()
    seg = _seg_ids(lod, t.device)
    pos = torch.arange(t.shape[0], device=t.device) - torch.tensor(lod[:-1], device=t.device)[seg]
    out[seg, pos] = t
    return _wrap(out), _wrap(torch.tensor(lens, dtype=torch.int64, device=t.device))


def sequence_unpad(x, length, name=None):
    t = _unwrap(x)
    lens = [int(v) for v in (_unwrap(length).reshape(-1).tolist() if isinstance(length, Tensor) else length)]
    rows = [t[i, :l] for i, l in enumerate(lens)]
    return with_lod(_wrap(torch.cat(rows, 0)), lengths_to_offsets(lens))


def sequence_reshape(input, new_dim):  # noqa: A002
    lod = get_lod(input)
    t = _unwrap(input)
    D = t.shape[1]
    new = [0]
    for l in offsets_to_lengths(lod):
        if (l * D) % new_dim:
            raise ValueError("sequence_reshape: sequence size not divisible by new_dim")
        new.append(new[-1] + l * D // new_dim)
    return with_lod(_wrap(t.reshape(-1, new_dim)), new)


def sequence_scatter(input, index, updates, name=None):  # noqa: A002
    """out = input; out[i, index_j] += updates_j for every element j of sequence i of index/updates."""
    lod = get_lod(index)
    t = _unwrap(input).clone()
    idx = _unwrap(index).reshape(-1).long()
    upd = _unwrap(updates).reshape(-1).to(t.dtype)
    seg = _seg_ids(lod, t.device)
    t.index_put_((seg, idx), upd, accumulate=True)
    return _wrap(t)


def sequence_enumerate(input, win_size, pad_value=0, name=None):  # noqa: A002
    """[N, win_size]: row t = ids t .. t+win_size-1 of t's sequence, pad_value past its end."""
    lod = get_lod(input)
    t = _unwrap(input).reshape(-1)
    N = t.shape[0]
    seg = _seg_ids(lod, t.device)
    ends = torch.tensor(lod[1:], device=t.device)[seg]
    pos = torch.arange(N, device=t.device)
    cols = []
    for j in range(win_size):
        src = pos + j
        cols.append(torch.where(src < ends, t[src.clamp(max=max(N - 1, 0))], torch.full_like(t, pad_value)))
    return with_lod(_wrap(torch.stack(cols, 1)), lod)


def row_conv_lod(x2, lod, w):
    """Lookahead convolution inside each sequence: out[t] = sum_j x[t+j] * w[j] (t+j in the same sequence)."""
    ctx = _context_rows(x2, lod, w.shape[0], 0)  # [N, k*D]
    return (ctx.reshape(x2.shape[0], w.shape[0], -1) * w.unsqueeze(0)).sum(1)
