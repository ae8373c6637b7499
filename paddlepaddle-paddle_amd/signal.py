"""paddle.signal (reference: python/paddle/signal.py — frame:30, overlap_add:145, stft:246,
istft:423)."""
import torch

from .core.tensor import _wrap, _unwrap


def frame(x, frame_length, hop_length, axis=-1, name=None):
    """Slices overlapping frames: axis=-1 → [..., frame_length, num_frames];
    axis=0 → [num_frames, frame_length, ...] (paddle layout)."""
    t = _unwrap(x)
    if axis not in (0, -1, t.dim() - 1):
        raise ValueError("frame: axis should be 0 or -1")
    if frame_length > t.shape[axis]:
        raise ValueError("frame_length exceeds the input length")
    if axis == 0:
        f = t.unfold(0, frame_length, hop_length)            # [n, ..., L]
        return _wrap(f.movedim(-1, 1))                        # [n, L, ...]
    f = t.unfold(-1, frame_length, hop_length)               # [..., n, L]
    return _wrap(f.transpose(-1, -2))                         # [..., L, n]


def overlap_add(x, hop_length, axis=-1, name=None):
    t = _unwrap(x)
    if axis == 0:
        t = t.movedim(0, -1).movedim(0, -2)  # [n, L, ...] -> [..., L, n]
    L, n = t.shape[-2], t.shape[-1]
    out_len = (n - 1) * hop_length + L
    lead = t.shape[:-2]
    flat = t.reshape(-1, L, n)
    out = torch.nn.functional.fold(flat, output_size=(1, out_len), kernel_size=(1, L), stride=(1, hop_length))
    out = out.reshape(*lead, out_len)
    if axis == 0:
        out = out.movedim(-1, 0)
    return _wrap(out)


def stft(x, n_fft, hop_length=None, win_length=None, window=None, center=True, pad_mode='reflect', normalized=False,
         onesided=True, name=None):
    t = _unwrap(x)
    w = _unwrap(window) if window is not None else None
    return _wrap(torch.stft(t, n_fft, hop_length, win_length, w, center, pad_mode, normalized,
                            onesided if not t.is_complex() else False, return_complex=True))


def istft(x, n_fft, hop_length=None, win_length=None, window=None, center=True, normalized=False, onesided=True,
          length=None, return_complex=False, name=None):
    w = _unwrap(window) if window is not None else None
    return _wrap(torch.istft(_unwrap(x), n_fft, hop_length, win_length, w, center, normalized, onesided, length,
                             return_complex))


__all__ = ['stft', 'istft']
