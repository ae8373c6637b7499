"""paddle.audio.features (reference: python/paddle/audio/features/layers.py — Spectrogram:24,
MelSpectrogram:106, LogMelSpectrogram:206, MFCC).  Inputs [B, T] waveforms; STFT on rocFFT."""
import torch

from ..nn.layer.layers import Layer
from ..core.tensor import _wrap, _unwrap
from . import functional as AF


class Spectrogram(Layer):
    def __init__(self, n_fft=512, hop_length=512, win_length=None, window='hann', power=1.0, center=True,
                 pad_mode='reflect', dtype='float32'):
        super().__init__()
        self.power = power
        self.n_fft = n_fft
        self.hop_length = hop_length
        self.win_length = win_length or n_fft
        self.center, self.pad_mode = center, pad_mode
        self.register_buffer('fft_window', AF.get_window(window, self.win_length, fftbins=True, dtype=dtype))

    def forward(self, x):
        t = _unwrap(x)
        w = self.fft_window._t.to(t.device)
        s = torch.stft(t, self.n_fft, self.hop_length, self.win_length, w, self.center, self.pad_mode,
                       return_complex=True)
        return _wrap(s.abs().pow(self.power))


class MelSpectrogram(Layer):
    def __init__(self, sr=22050, n_fft=2048, hop_length=512, win_length=None, window='hann', power=2.0, center=True,
                 pad_mode='reflect', n_mels=64, f_min=50.0, f_max=None, htk=False, norm='slaney', dtype='float32'):
        super().__init__()
        self._spectrogram = Spectrogram(n_fft, hop_length, win_length, window, power, center, pad_mode, dtype)
        self.n_mels, self.f_min, self.f_max = n_mels, f_min, f_max
        self.register_buffer('fbank_matrix', AF.compute_fbank_matrix(sr, n_fft, n_mels, f_min, f_max, htk, norm,
                                                                     dtype))

    def forward(self, x):
        spect = _unwrap(self._spectrogram(x))
        return _wrap(torch.matmul(self.fbank_matrix._t.to(spect.device), spect))


class LogMelSpectrogram(Layer):
    def __init__(self, sr=22050, n_fft=512, hop_length=None, win_length=None, window='hann', power=2.0, center=True,
                 pad_mode='reflect', n_mels=64, f_min=50.0, f_max=None, htk=False, norm='slaney', ref_value=1.0,
                 amin=1e-10, top_db=None, dtype='float32'):
        super().__init__()
        self._melspectrogram = MelSpectrogram(sr, n_fft, hop_length, win_length, window, power, center, pad_mode,
                                              n_mels, f_min, f_max, htk, norm, dtype)
        self.ref_value, self.amin, self.top_db = ref_value, amin, top_db

    def forward(self, x):
        return AF.power_to_db(self._melspectrogram(x), self.ref_value, self.amin, self.top_db)


class MFCC(Layer):
    def __init__(self, sr=22050, n_mfcc=40, n_fft=512, hop_length=None, win_length=None, window='hann', power=2.0,
                 center=True, pad_mode='reflect', n_mels=64, f_min=50.0, f_max=None, htk=False, norm='slaney',
                 ref_value=1.0, amin=1e-10, top_db=None, dtype='float32'):
        super().__init__()
        if n_mfcc > n_mels:
            raise ValueError("n_mfcc cannot be larger than n_mels")
        self._log_melspectrogram = LogMelSpectrogram(sr, n_fft, hop_length, win_length, window, power, center,
                                                     pad_mode, n_mels, f_min, f_max, htk, norm, ref_value, amin,
                                                     top_db, dtype)
        self.register_buffer('dct_matrix', AF.create_dct(n_mfcc, n_mels, 'ortho', dtype))

    def forward(self, x):
        lm = _unwrap(self._log_melspectrogram(x))               # [B, n_mels, frames]
        return _wrap(torch.matmul(lm.transpose(-1, -2), self.dct_matrix._t.to(lm.device)).transpose(-1, -2))


__all__ = ['LogMelSpectrogram', 'MelSpectrogram', 'MFCC', 'Spectrogram']
