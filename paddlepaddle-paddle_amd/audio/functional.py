"""paddle.audio.functional (reference: python/paddle/audio/functional/functional.py, window.py).
Slaney / HTK mel scales, filter banks, dB conversion, DCT and window functions on device."""
import math

import numpy as np
import torch

from ..core.tensor import Tensor, _wrap, _unwrap
from ..core.dtype import to_torch_dtype


def _dev():
    from ..core.place import current_device
    return current_device()


def hz_to_mel(freq, htk=False):
    is_t = isinstance(freq, Tensor)
    f = _unwrap(freq) if is_t else freq
    if htk:
        return _wrap(2595.0 * torch.log10(1.0 + f / 700.0)) if is_t else 2595.0 * math.log10(1.0 + f / 700.0)
    f_sp = 200.0 / 3
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, math.log(6.4) / 27.0
    if is_t:
        mels = f / f_sp
        log_part = min_log_mel + torch.log(f / min_log_hz + 1e-10) / logstep
        return _wrap(torch.where(f >= min_log_hz, log_part, mels))
    if f >= min_log_hz:
        return min_log_mel + math.log(f / min_log_hz + 1e-10) / logstep
    return f / f_sp


def mel_to_hz(mel, htk=False):
    is_t = isinstance(mel, Tensor)
    m = _unwrap(mel) if is_t else mel
    if htk:
        return _wrap(700.0 * (10.0 ** (m / 2595.0) - 1.0)) if is_t else 700.0 * (10.0 ** (m / 2595.0) - 1.0)
    f_sp = 200.0 / 3
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, math.log(6.4) / 27.0
    if is_t:
        return _wrap(torch.where(m >= min_log_mel, min_log_hz * torch.exp(logstep * (m - min_log_mel)), f_sp * m))
    if m >= min_log_mel:
        return min_log_hz * math.exp(logstep * (m - min_log_mel))
    return f_sp * m


def mel_frequencies(n_mels=64, f_min=0.0, f_max=11025.0, htk=False, dtype='float32'):
    lo, hi = hz_to_mel(f_min, htk), hz_to_mel(f_max, htk)
    mels = torch.linspace(lo, hi, n_mels, dtype=to_torch_dtype(dtype), device=_dev())
    return mel_to_hz(_wrap(mels), htk)


def fft_frequencies(sr, n_fft, dtype='float32'):
    return _wrap(torch.linspace(0, float(sr) / 2, int(1 + n_fft // 2), dtype=to_torch_dtype(dtype), device=_dev()))


def compute_fbank_matrix(sr, n_fft, n_mels=64, f_min=0.0, f_max=None, htk=False, norm='slaney', dtype='float32'):
    if f_max is None:
        f_max = float(sr) / 2
    fftfreqs = _unwrap(fft_frequencies(sr, n_fft, dtype))
    mel_f = _unwrap(mel_frequencies(n_mels + 2, f_min, f_max, htk, dtype))
    fdiff = mel_f[1:] - mel_f[:-1]
    ramps = mel_f.unsqueeze(1) - fftfreqs.unsqueeze(0)
    lower = -ramps[:n_mels] / fdiff[:n_mels].unsqueeze(1)
    upper = ramps[2:n_mels + 2] / fdiff[1:n_mels + 1].unsqueeze(1)
    weights = torch.clamp(torch.minimum(lower, upper), min=0)
    if norm == 'slaney':
        enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
        weights = weights * enorm.unsqueeze(1)
    elif isinstance(norm, (int, float)):
        weights = torch.nn.functional.normalize(weights, p=norm, dim=-1)
    return _wrap(weights)


def power_to_db(spect, ref_value=1.0, amin=1e-10, top_db=80.0):
    if amin <= 0:
        raise ValueError("amin must be strictly positive")
    if ref_value <= 0:
        raise ValueError("ref_value must be strictly positive")
    s = _unwrap(spect)
    log_spec = 10.0 * torch.log10(torch.clamp(s, min=amin))
    log_spec = log_spec - 10.0 * math.log10(max(ref_value, amin))
    if top_db is not None:
        if top_db < 0:
            raise ValueError("top_db must be non-negative")
        log_spec = torch.maximum(log_spec, log_spec.max() - top_db)
    return _wrap(log_spec)


def create_dct(n_mfcc, n_mels, norm='ortho', dtype='float32'):
    dt = to_torch_dtype(dtype)
    n = torch.arange(n_mels, dtype=dt, device=_dev())
    k = torch.arange(n_mfcc, dtype=dt, device=_dev()).unsqueeze(1)
    dct = torch.cos(math.pi / float(n_mels) * (n + 0.5) * k)
    if norm is None:
        dct = dct * 2.0
    else:
        dct[0] *= 1.0 / math.sqrt(2.0)
        dct = dct * math.sqrt(2.0 / float(n_mels))
    return _wrap(dct.T)


def _general_cosine(M, a, sym):
    M_ext = M + 1 if not sym else M
    fac = np.linspace(-np.pi, np.pi, M_ext)
    w = np.zeros(M_ext)
    for k, ak in enumerate(a):
        w += ak * np.cos(k * fac)
    return w[:M] if not sym else w


def get_window(window, win_length, fftbins=True, dtype='float64'):
    """hann, hamming, blackman, bohman, cosine, triang, gaussian (std), exponential, tukey, taylor."""
    sym = not fftbins
    params = ()
    if isinstance(window, tuple):
        window, params = window[0], window[1:]
    M = win_length
    Mx = M + 1 if not sym else M
    n = np.arange(Mx)
    if window in ('hann', 'hanning'):
        w = _general_cosine(M, [0.5, 0.5], sym)
    elif window == 'hamming':
        w = _general_cosine(M, [0.54, 0.46], sym)
    elif window == 'blackman':
        w = _general_cosine(M, [0.42, 0.50, 0.08], sym)
    elif window == 'cosine':
        w = np.sin(np.pi / Mx * (n + 0.5))[:M]
    elif window == 'triang':
        w = np.bartlett(Mx + 2)[1:-1][:M] if Mx % 2 else 1 - np.abs((2 * n - Mx + 1) / Mx)
        w = w[:M]
    elif window == 'bohman':
        fac = np.abs(np.linspace(-1, 1, Mx)[1:-1])
        w = np.r_[0, (1 - fac) * np.cos(np.pi * fac) + 1.0 / np.pi * np.sin(np.pi * fac), 0][:M]
    elif window == 'gaussian':
        std = params[0] if params else 1.0
        w = np.exp(-0.5 * ((n - (Mx - 1) / 2.0) / std) ** 2)[:M]
    elif window == 'exponential':
        tau = params[-1] if params else 1.0
        w = np.exp(-np.abs(n - (Mx - 1) / 2.0) / tau)[:M]
    elif window == 'tukey':
        alpha = params[0] if params else 0.5
        w = np.ones(Mx)
        width = int(np.floor(alpha * (Mx - 1) / 2.0))
        n1 = n[:width + 1]
        w[:width + 1] = 0.5 * (1 + np.cos(np.pi * (-1 + 2.0 * n1 / alpha / (Mx - 1))))
        w[Mx - width - 1:] = w[:width + 1][::-1]
        w = w[:M]
    else:
        raise ValueError(f"unsupported window {window}")
    return _wrap(torch.tensor(np.asarray(w), dtype=to_torch_dtype(dtype), device=_dev()))


__all__ = ['compute_fbank_matrix', 'create_dct', 'fft_frequencies', 'hz_to_mel', 'mel_frequencies', 'mel_to_hz',
           'power_to_db', 'get_window']
