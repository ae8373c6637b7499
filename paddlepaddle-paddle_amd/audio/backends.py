"""Audio IO (reference: python/paddle/audio/backends/{wave_backend,init_backend}.py): WAV via the
standard-library ``wave`` module (PCM 8/16/32-bit)."""
import wave

import numpy as np
import torch

from ..core.tensor import _wrap, _unwrap


class AudioInfo:
    def __init__(self, sample_rate, num_frames, num_channels, bits_per_sample, encoding):
        self.sample_rate, self.num_frames, self.num_channels = sample_rate, num_frames, num_channels
        self.bits_per_sample, self.encoding = bits_per_sample, encoding


def list_available_backends():
    return ['wave_backend']


def get_current_backend():
    return 'wave_backend'


def set_backend(backend_name):
    if backend_name != 'wave_backend':
        raise NotImplementedError("only the builtin wave backend is available")


def info(filepath):
    with wave.open(str(filepath), 'rb') as f:
        return AudioInfo(f.getframerate(), f.getnframes(), f.getnchannels(), f.getsampwidth() * 8, 'PCM_S')


_DT = {1: np.uint8, 2: np.int16, 4: np.int32}


def load(filepath, frame_offset=0, num_frames=-1, normalize=True, channels_first=True):
    with wave.open(str(filepath), 'rb') as f:
        sr, ch, sw = f.getframerate(), f.getnchannels(), f.getsampwidth()
        f.setpos(frame_offset)
        n = f.getnframes() - frame_offset if num_frames < 0 else num_frames
        raw = f.readframes(n)
    a = np.frombuffer(raw, dtype=_DT[sw]).reshape(-1, ch)
    if normalize:
        if sw == 1:
            a = (a.astype(np.float32) - 128) / 128.0
        else:
            a = a.astype(np.float32) / float(2 ** (8 * sw - 1))
    t = torch.from_numpy(np.ascontiguousarray(a.T if channels_first else a))
    return _wrap(t), sr


def save(filepath, src, sample_rate, channels_first=True, encoding=None, bits_per_sample=16):
    a = _unwrap(src).detach().cpu().numpy()
    if channels_first:
        a = a.T
    if a.ndim == 1:
        a = a[:, None]
    sw = bits_per_sample // 8
    if np.issubdtype(a.dtype, np.floating):
        a = np.clip(a, -1, 1) * (2 ** (8 * sw - 1) - 1)
    with wave.open(str(filepath), 'wb') as f:
        f.setnchannels(a.shape[1])
        f.setsampwidth(sw)
        f.setframerate(int(sample_rate))
        f.writeframes(a.astype(_DT[sw]).tobytes())
