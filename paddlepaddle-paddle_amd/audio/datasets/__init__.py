"""paddle.audio.datasets (reference: python/paddle/audio/datasets/{dataset,esc50,tess}.py).

Local files only: the archives are looked up under ``DATA_HOME`` (``$PADDLE_DATA_HOME`` or
``~/.cache/paddle/dataset``) or an explicit ``data_home=``; nothing is downloaded.
"""
import collections
import os

from ...io.dataset import Dataset

__all__ = ['ESC50', 'TESS']

DATA_HOME = os.environ.get('PADDLE_DATA_HOME', os.path.join(os.path.expanduser('~'), '.cache', 'paddle', 'dataset'))


def _feat_funcs():
    from ..features import MFCC, LogMelSpectrogram, MelSpectrogram, Spectrogram
    return {'raw': None, 'melspectrogram': MelSpectrogram, 'mfcc': MFCC, 'logmelspectrogram': LogMelSpectrogram,
            'spectrogram': Spectrogram}


class AudioClassificationDataset(Dataset):
    """(feature, label) pairs of audio files; features computed on access by paddle.audio.features."""

    def __init__(self, files, labels, feat_type='raw', sample_rate=None, **kwargs):
        super().__init__()
        if feat_type not in _feat_funcs():
            raise RuntimeError(f"Unknown feat_type: {feat_type}, it must be one in {list(_feat_funcs())}")
        self.files, self.labels = files, labels
        self.feat_type, self.sample_rate = feat_type, sample_rate
        self.feat_config = kwargs

    def _convert_to_record(self, idx):
        import paddle
        from ..backends import load
        file, label = self.files[idx], self.labels[idx]
        waveform, sample_rate = load(file)
        self.sample_rate = sample_rate
        if len(waveform.shape) == 2:
            waveform = waveform.squeeze(0)
        waveform = paddle.to_tensor(waveform, dtype='float32')
        f = _feat_funcs()[self.feat_type]
        if f is not None:
            x = waveform.unsqueeze(0)
            ext = f(**self.feat_config) if self.feat_type == 'spectrogram' else f(sr=self.sample_rate,
                                                                                   **self.feat_config)
            feat = ext(x).squeeze(0)
        else:
            feat = waveform
        return feat, label

    def __getitem__(self, idx):
        return self._convert_to_record(idx)

    def __len__(self):
        return len(self.files)


def _need(path, what):
    if not os.path.exists(path):
        raise RuntimeError(f"{what} not found at {path}: place the extracted archive there "
                           f"(no network access, nothing is downloaded)")


class ESC50(AudioClassificationDataset):
    """ESC-50: 2000 five-second environmental recordings, 50 classes, 5 folds (``split`` = dev fold)."""

    label_list = [
        'Dog', 'Rooster', 'Pig', 'Cow', 'Frog', 'Cat', 'Hen', 'Insects (flying)', 'Sheep', 'Crow',
        'Rain', 'Sea waves', 'Crackling fire', 'Crickets', 'Chirping birds', 'Water drops', 'Wind', 'Pouring water',
        'Toilet flush', 'Thunderstorm',
        'Crying baby', 'Sneezing', 'Clapping', 'Breathing', 'Coughing', 'Footsteps', 'Laughing', 'Brushing teeth',
        'Snoring', 'Drinking, sipping',
        'Door knock', 'Mouse click', 'Keyboard typing', 'Door, wood creaks', 'Can opening', 'Washing machine',
        'Vacuum cleaner', 'Clock alarm', 'Clock tick', 'Glass breaking',
        'Helicopter', 'Chainsaw', 'Siren', 'Car horn', 'Engine', 'Train', 'Church bells', 'Airplane', 'Fireworks',
        'Hand saw']
    meta = os.path.join('ESC-50-master', 'meta', 'esc50.csv')
    meta_info = collections.namedtuple('META_INFO',
                                       ('filename', 'fold', 'target', 'category', 'esc10', 'src_file', 'take'))
    audio_path = os.path.join('ESC-50-master', 'audio')

    def __init__(self, mode='train', split=1, feat_type='raw', archive=None, data_home=None, **kwargs):
        assert split in range(1, 6), f'The selected split should be integer, and 1 <= split <= 5, but got {split}'
        self.data_home = data_home or DATA_HOME
        files, labels = self._get_data(mode, split)
        super().__init__(files=files, labels=labels, feat_type=feat_type, **kwargs)

    def _get_meta_info(self):
        with open(os.path.join(self.data_home, self.meta)) as rf:
            return [self.meta_info(*line.strip().split(',')) for line in rf.readlines()[1:] if line.strip()]

    def _get_data(self, mode, split):
        _need(os.path.join(self.data_home, self.meta), 'ESC-50 metadata')
        files, labels = [], []
        for s in self._get_meta_info():
            if (mode == 'train') == (int(s.fold) != split):
                files.append(os.path.join(self.data_home, self.audio_path, s.filename))
                labels.append(int(s.target))
        return files, labels


class TESS(AudioClassificationDataset):
    """Toronto emotional speech set: 2800 clips, 7 emotions; ``n_folds`` round-robin folds."""

    label_list = ['angry', 'disgust', 'fear', 'happy', 'neutral', 'ps', 'sad']
    meta_info = collections.namedtuple('META_INFO', ('speaker', 'word', 'emotion'))
    audio_path = 'TESS_Toronto_emotional_speech_set'

    def __init__(self, mode='train', n_folds=5, split=1, feat_type='raw', archive=None, data_home=None, **kwargs):
        assert isinstance(n_folds, int) and n_folds >= 1, f'the n_folds should be integer and n_folds >= 1, ' \
                                                          f'but got {n_folds}'
        assert split in range(1, n_folds + 1), \
            f'The selected split should be integer and should be 1 <= split <= {n_folds}, but got {split}'
        self.data_home = data_home or DATA_HOME
        files, labels = self._get_data(mode, n_folds, split)
        super().__init__(files=files, labels=labels, feat_type=feat_type, **kwargs)

    def _get_data(self, mode, n_folds, split):
        root = os.path.join(self.data_home, self.audio_path)
        _need(root, 'TESS audio directory')
        wav = sorted(os.path.join(r, f) for r, _, fs in os.walk(root) for f in fs if f.endswith('.wav'))
        files, labels = [], []
        for idx, f in enumerate(wav):
            emotion = self.meta_info(*os.path.basename(f)[:-4].split('_')).emotion
            fold = idx % n_folds + 1
            if (mode == 'train') == (fold != split):
                files.append(f)
                labels.append(self.label_list.index(emotion))
        return files, labels
