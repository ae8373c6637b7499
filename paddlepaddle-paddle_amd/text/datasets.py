"""paddle.text.datasets: the NLP corpora, parsed from local archives (no downloads).

Reference: python/paddle/text/datasets/{imdb,imikolov,movielens,conll05,wmt14,wmt16,
uci_housing}.py.  Same constructor arguments and the same per-sample arrays; ``data_file`` (and the
dictionary files of Conll05st) must point at local copies of the published archives:

  Imdb       aclImdb_v1.tar.gz       (aclImdb/{train,test}/{pos,neg}/*.txt)
  Imikolov   simple-examples.tgz     (./simple-examples/data/ptb.{train,valid,test}.txt)
  Movielens  ml-1m.zip               (ml-1m/{movies,users,ratings}.dat)
  Conll05st  conll05st-tests.tar.gz  (test.wsj words/props, gzip) + word/verb/target dicts
  WMT14      wmt_shrinked_data.tgz   (*src.dict, *trg.dict, {mode}/{mode} tab-separated pairs)
  WMT16      wmt16.tar.gz            (wmt16/{train,test,val} tab-separated en/de pairs)
"""
import collections
import gzip
import os
import re
import string
import tarfile
import zipfile

import numpy as np

from ..io.dataset import Dataset

__all__ = ['Conll05st', 'Imdb', 'Imikolov', 'Movielens', 'UCIHousing', 'WMT14', 'WMT16']

DATA_HOME = os.environ.get('PADDLE_DATA_HOME', os.path.join(os.path.expanduser('~'), '.cache', 'paddle', 'dataset'))


def _local(data_file, what, download=True):
    if data_file is None:
        raise RuntimeError(f"{what}: no network access, nothing is downloaded; pass data_file= pointing at a local "
                           f"copy of the archive")
    if not os.path.exists(data_file):
        raise RuntimeError(f"{what}: {data_file} not found")
    return data_file


def _mode(mode, allowed):
    m = mode.lower()
    assert m in allowed, f"mode should be {', '.join(repr(a) for a in allowed)}, but got {mode}"
    return m


def _ranked_vocab(freq, cutoff):
    """word -> id by descending frequency (ties by word), words seen more than ``cutoff`` times,
    '<unk>' last."""
    kept = sorted(((w, c) for w, c in freq.items() if c > cutoff), key=lambda x: (-x[1], x[0]))
    vocab = {w: i for i, (w, _) in enumerate(kept)}
    vocab['<unk>'] = len(kept)
    return vocab


class Imdb(Dataset):
    """Sentiment classification: (word ids of a review, [label]) with label 0 = pos, 1 = neg; the
    vocabulary counts train + test words over ``cutoff``."""

    _PUNCT = string.punctuation.encode('latin-1')

    def __init__(self, data_file=None, mode='train', cutoff=150, download=True):
        self.mode = _mode(mode, ('train', 'test'))
        self.data_file = _local(data_file, 'Imdb')
        docs = self._read(re.compile(r"aclImdb/(train|test)/(pos|neg)/.*\.txt$"))
        freq = collections.Counter(w for _, d in docs for w in d)
        self.word_idx = _ranked_vocab(freq, cutoff)
        unk = self.word_idx['<unk>']
        self.docs, self.labels = [], []
        for want, label in (('pos', 0), ('neg', 1)):
            pat = re.compile(fr"aclImdb/{self.mode}/{want}/.*\.txt$")
            for name, d in docs:
                if pat.match(name):
                    self.docs.append([self.word_idx.get(w, unk) for w in d])
                    self.labels.append(label)

    def _read(self, pattern):
        out = []
        with tarfile.open(self.data_file) as tf:
            for m in tf:
                if m.isfile() and pattern.match(m.name):
                    txt = tf.extractfile(m).read().rstrip(b'\n\r').translate(None, self._PUNCT).lower()
                    out.append((m.name, txt.split()))
        return out

    def __getitem__(self, idx):
        return np.array(self.docs[idx]), np.array([self.labels[idx]])

    def __len__(self):
        return len(self.docs)


class Imikolov(Dataset):
    """Penn Treebank language modelling: NGRAM windows of ``window_size`` ids, or SEQ
    (<s> + ids, ids + <e>) pairs; vocabulary from train + valid words over ``min_word_freq``."""

    def __init__(self, data_file=None, data_type='NGRAM', window_size=-1, mode='train', min_word_freq=50,
                 download=True):
        self.data_type = data_type.upper()
        assert self.data_type in ('NGRAM', 'SEQ'), f"data type should be 'NGRAM', 'SEQ', but got {data_type}"
        self.mode = _mode(mode, ('train', 'test'))
        self.window_size, self.min_word_freq = window_size, min_word_freq
        self.data_file = _local(data_file, 'Imikolov')
        with tarfile.open(self.data_file) as tf:
            freq = collections.Counter()
            for split in ('train', 'valid'):
                for line in self._lines(tf, split):
                    freq.update(line.split())
                    freq['<s>'] += 1
                    freq['<e>'] += 1
            freq.pop('<unk>', None)
            self.word_idx = _ranked_vocab(freq, min_word_freq)
            unk = self.word_idx['<unk>']
            self.data = []
            for line in self._lines(tf, self.mode):
                words = line.split()
                if self.data_type == 'NGRAM':
                    assert self.window_size > -1, 'Invalid gram length'
                    ids = [self.word_idx.get(w, unk) for w in ['<s>'] + words + ['<e>']]
                    if len(ids) >= self.window_size:
                        self.data.extend(tuple(ids[i - self.window_size:i])
                                         for i in range(self.window_size, len(ids) + 1))
                else:
                    ids = [self.word_idx.get(w, unk) for w in words]
                    src = [self.word_idx['<s>']] + ids
                    if self.window_size > 0 and len(src) > self.window_size:
                        continue
                    self.data.append((src, ids + [self.word_idx['<e>']]))

    @staticmethod
    def _lines(tf, split):
        for m in tf.getmembers():
            if m.isfile() and m.name.lstrip('./').endswith(f'simple-examples/data/ptb.{split}.txt'):
                return [ln.decode('utf-8', 'ignore').strip() for ln in tf.extractfile(m)]
        raise RuntimeError(f"Imikolov: ptb.{split}.txt not in the archive")

    def __getitem__(self, idx):
        return tuple(np.array(d) for d in self.data[idx])

    def __len__(self):
        return len(self.data)


_AGES = [1, 18, 25, 35, 45, 50, 56]


class MovieInfo:
    def __init__(self, index, categories, title):
        self.index, self.categories, self.title = int(index), categories, title

    def value(self, categories_dict, movie_title_dict):
        return [[self.index], [categories_dict[c] for c in self.categories],
                [movie_title_dict[w.lower()] for w in self.title.split()]]

    def __repr__(self):
        return f"<MovieInfo id({self.index}), title({self.title}), categories({self.categories})>"


class UserInfo:
    def __init__(self, index, gender, age, job_id):
        self.index, self.is_male, self.age, self.job_id = int(index), gender == 'M', _AGES.index(int(age)), int(job_id)

    def value(self):
        return [[self.index], [0 if self.is_male else 1], [self.age], [self.job_id]]

    def __repr__(self):
        return f"<UserInfo id({self.index}), gender({'M' if self.is_male else 'F'}), age({_AGES[self.age]}), " \
               f"job({self.job_id})>"


class Movielens(Dataset):
    """MovieLens-1M ratings: user id / gender / age bucket / job, movie id / category ids / title
    word ids, and the rating mapped to 2r - 5; ``test_ratio`` of the ratings (seeded) form the
    test split."""

    def __init__(self, data_file=None, mode='train', test_ratio=0.1, rand_seed=0, download=True):
        self.mode = _mode(mode, ('train', 'test'))
        self.data_file = _local(data_file, 'Movielens')
        self.test_ratio, self.rand_seed = test_ratio, rand_seed
        rng = np.random.RandomState(rand_seed)
        title_re = re.compile(r'^(.*)\((\d+)\)$')
        self.movie_info, self.user_info = {}, {}
        words, cats = [], []
        with zipfile.ZipFile(self.data_file) as z:
            for line in z.open('ml-1m/movies.dat'):
                mid, title, cs = line.decode('latin').strip().split('::')
                cs = cs.split('|')
                title = title_re.match(title).group(1)
                self.movie_info[int(mid)] = MovieInfo(mid, cs, title)
                cats.extend(c for c in cs if c not in cats)
                words.extend(w.lower() for w in title.split())
            self.movie_title_dict = {w: i for i, w in enumerate(dict.fromkeys(words))}
            self.categories_dict = {c: i for i, c in enumerate(cats)}
            for line in z.open('ml-1m/users.dat'):
                uid, gender, age, job, _ = line.decode('latin').strip().split('::')
                self.user_info[int(uid)] = UserInfo(uid, gender, age, job)
            self.data = []
            want_test = self.mode == 'test'
            for line in z.open('ml-1m/ratings.dat'):
                if (rng.random_sample() < test_ratio) != want_test:
                    continue
                uid, mid, rating, _ = line.decode('latin').strip().split('::')
                usr, mov = self.user_info[int(uid)], self.movie_info[int(mid)]
                self.data.append(usr.value() + mov.value(self.categories_dict, self.movie_title_dict) +
                                 [[float(rating) * 2 - 5.0]])

    def __getitem__(self, idx):
        return tuple(np.array(d) for d in self.data[idx])

    def __len__(self):
        return len(self.data)


class Conll05st(Dataset):
    """CoNLL-2005 semantic role labelling (test.wsj): per (sentence, predicate): word ids, the five
    context-word ids around the predicate broadcast over the sentence, predicate ids, the
    context mark and BIO label ids."""

    UNK_IDX = 0

    def __init__(self, data_file=None, word_dict_file=None, verb_dict_file=None, target_dict_file=None,
                 emb_file=None, download=True):
        self.data_file = _local(data_file, 'Conll05st')
        self.word_dict = self._load_dict(_local(word_dict_file, 'Conll05st word dict'))
        self.predicate_dict = self._load_dict(_local(verb_dict_file, 'Conll05st verb dict'))
        self.label_dict = self._load_label_dict(_local(target_dict_file, 'Conll05st target dict'))
        self.emb_file = emb_file
        self.sentences, self.predicates, self.labels = [], [], []
        self._load()

    @staticmethod
    def _load_dict(fn):
        with open(fn) as f:
            return {line.strip(): i for i, line in enumerate(f)}

    @staticmethod
    def _load_label_dict(fn):
        tags = []
        with open(fn) as f:
            for line in f:
                line = line.strip()
                if line[:2] in ('B-', 'I-') and line[2:] not in tags:
                    tags.append(line[2:])
        d = {}
        for t in tags:
            d['B-' + t] = len(d)
            d['I-' + t] = len(d)
        d['O'] = len(d)
        return d

    @staticmethod
    def _bio(column):
        out, tag, open_ = [], 'O', False
        for l in column:
            if l == '*':
                out.append('I-' + tag if open_ else 'O')
            elif l == '*)':
                out.append('I-' + tag)
                open_ = False
            elif '(' in l:
                tag = l[1:l.find('*')]
                out.append('B-' + tag)
                open_ = ')' not in l
            else:
                raise RuntimeError(f'Unexpected label: {l}')
        return out

    def _load(self):
        with tarfile.open(self.data_file) as tf:
            words = tf.extractfile("conll05st-release/test.wsj/words/test.wsj.words.gz")
            props = tf.extractfile("conll05st-release/test.wsj/props/test.wsj.props.gz")
            with gzip.GzipFile(fileobj=words) as wf, gzip.GzipFile(fileobj=props) as pf:
                sent, rows = [], []
                for w, p in zip(wf, pf):
                    w, cols = w.strip().decode(), p.strip().decode().split()
                    if cols:
                        sent.append(w)
                        rows.append(cols)
                        continue
                    if rows:
                        columns = list(zip(*rows))
                        verbs = [x for x in columns[0] if x != '-']
                        for i, col in enumerate(columns[1:]):
                            self.sentences.append(sent)
                            self.predicates.append(verbs[i])
                            self.labels.append(self._bio(col))
                    sent, rows = [], []

    def __getitem__(self, idx):
        sentence, predicate, labels = self.sentences[idx], self.predicates[idx], self.labels[idx]
        n = len(sentence)
        v = labels.index('B-V')
        mark = [0] * n
        ctx = {}
        for off, key in ((-2, 'n2'), (-1, 'n1'), (0, '0'), (1, 'p1'), (2, 'p2')):
            j = v + off
            if 0 <= j < n:
                mark[j] = 1
                ctx[key] = sentence[j]
            else:
                ctx[key] = 'bos' if off < 0 else 'eos'
        wd = self.word_dict
        ids = lambda w: [wd.get(w, self.UNK_IDX)] * n  # noqa: E731
        return (np.array([wd.get(w, self.UNK_IDX) for w in sentence]), np.array(ids(ctx['n2'])),
                np.array(ids(ctx['n1'])), np.array(ids(ctx['0'])), np.array(ids(ctx['p1'])),
                np.array(ids(ctx['p2'])), np.array([self.predicate_dict.get(predicate)] * n), np.array(mark),
                np.array([self.label_dict.get(t) for t in labels]))

    def __len__(self):
        return len(self.sentences)

    def get_dict(self):
        return self.word_dict, self.predicate_dict, self.label_dict

    def get_embedding(self):
        return self.emb_file


_START, _END, _UNK = '<s>', '<e>', '<unk>'


class WMT14(Dataset):
    """WMT'14 en-fr (shrinked): (<s> src <e> ids, <s> trg ids, trg <e> ids), the first
    ``dict_size`` entries of the shipped dictionaries; pairs longer than 80 ids are dropped."""

    UNK_IDX = 2

    def __init__(self, data_file=None, mode='train', dict_size=-1, download=True):
        self.mode = _mode(mode, ('train', 'test', 'gen'))
        self.data_file = _local(data_file, 'WMT14')
        assert dict_size > 0, "dict_size should be set as positive number"
        self.dict_size = dict_size
        self.src_ids, self.trg_ids, self.trg_ids_next = [], [], []
        with tarfile.open(self.data_file) as tf:
            members = tf.getmembers()

            def vocab(suffix):
                m = [x for x in members if x.name.endswith(suffix)]
                assert len(m) == 1, suffix
                out = {}
                for i, line in enumerate(tf.extractfile(m[0])):
                    if i >= dict_size:
                        break
                    out[line.strip().decode()] = i
                return out
            self.src_dict, self.trg_dict = vocab('src.dict'), vocab('trg.dict')
            for m in members:
                if not m.name.endswith(f"{self.mode}/{self.mode}"):
                    continue
                for line in tf.extractfile(m):
                    parts = line.decode().strip().split('\t')
                    if len(parts) != 2:
                        continue
                    src = [self.src_dict.get(w, self.UNK_IDX) for w in [_START] + parts[0].split() + [_END]]
                    trg = [self.trg_dict.get(w, self.UNK_IDX) for w in parts[1].split()]
                    if len(src) > 80 or len(trg) > 80:
                        continue
                    self.src_ids.append(src)
                    self.trg_ids.append([self.trg_dict[_START]] + trg)
                    self.trg_ids_next.append(trg + [self.trg_dict[_END]])

    def __getitem__(self, idx):
        return np.array(self.src_ids[idx]), np.array(self.trg_ids[idx]), np.array(self.trg_ids_next[idx])

    def __len__(self):
        return len(self.src_ids)

    def get_dict(self, reverse=False):
        s, t = self.src_dict, self.trg_dict
        if reverse:
            s, t = {v: k for k, v in s.items()}, {v: k for k, v in t.items()}
        return s, t


class WMT16(Dataset):
    """WMT'16 Multi30k en-de: dictionaries of the ``*_dict_size`` most frequent train words (after
    <s>, <e>, <unk>), cached as DATA_HOME/wmt16/{lang}_{size}.dict like the reference."""

    TOTAL_EN_WORDS, TOTAL_DE_WORDS = 11250, 19220

    def __init__(self, data_file=None, mode='train', src_dict_size=-1, trg_dict_size=-1, lang='en', download=True,
                 dict_dir=None):
        self.mode = _mode(mode, ('train', 'test', 'val'))
        self.data_file = _local(data_file, 'WMT16')
        assert src_dict_size > 0 and trg_dict_size > 0, "dict_size should be set as positive number"
        self.lang = lang
        self.dict_dir = dict_dir or os.path.join(DATA_HOME, 'wmt16')
        en = lang == 'en'
        self.src_dict_size = min(src_dict_size, self.TOTAL_EN_WORDS if en else self.TOTAL_DE_WORDS)
        self.trg_dict_size = min(trg_dict_size, self.TOTAL_DE_WORDS if en else self.TOTAL_EN_WORDS)
        self.src_dict = self._load_dict(lang, src_dict_size)
        self.trg_dict = self._load_dict('de' if en else 'en', trg_dict_size)
        start, end, unk = self.src_dict[_START], self.src_dict[_END], self.src_dict[_UNK]
        sc = 0 if en else 1
        self.src_ids, self.trg_ids, self.trg_ids_next = [], [], []
        for a, b in self._pairs(self.mode):
            s, t = (a, b) if sc == 0 else (b, a)
            self.src_ids.append([start] + [self.src_dict.get(w, unk) for w in s.split()] + [end])
            tids = [self.trg_dict.get(w, unk) for w in t.split()]
            self.trg_ids.append([start] + tids)
            self.trg_ids_next.append(tids + [end])

    def _pairs(self, split):
        with tarfile.open(self.data_file) as tf:
            for line in tf.extractfile(f"wmt16/{split}"):
                parts = line.decode().strip().split('\t')
                if len(parts) == 2:
                    yield parts[0], parts[1]

    def _load_dict(self, lang, size):
        path = os.path.join(self.dict_dir, f"{lang}_{size}.dict")
        ok = False
        if os.path.exists(path):
            with open(path, 'rb') as f:
                ok = len(f.readlines()) == size
        if not ok:
            col = 0 if lang == 'en' else 1
            freq = collections.Counter()
            for pair in self._pairs('train'):
                freq.update(pair[col].split())
            os.makedirs(self.dict_dir, exist_ok=True)
            ranked = [w for w, _ in sorted(freq.items(), key=lambda x: x[1], reverse=True)][:max(size - 3, 0)]
            with open(path, 'wb') as f:
                f.write('\n'.join([_START, _END, _UNK] + ranked).encode() + b'\n')
        with open(path, 'rb') as f:
            return {line.strip().decode(): i for i, line in enumerate(f)}

    def __getitem__(self, idx):
        return np.array(self.src_ids[idx]), np.array(self.trg_ids[idx]), np.array(self.trg_ids_next[idx])

    def __len__(self):
        return len(self.src_ids)

    def get_dict(self, lang, reverse=False):
        d = self.src_dict if lang == self.lang else self.trg_dict
        return {v: k for k, v in d.items()} if reverse else d


class UCIHousing(Dataset):
    """Boston housing regression (13 normalised features -> price) from the whitespace table
    ``housing.data``; first 80 % train, the rest test."""

    def __init__(self, data_file=None, mode='train', download=True):
        self.mode = _mode(mode, ('train', 'test'))
        data = np.loadtxt(_local(data_file, 'UCIHousing')).astype('float32')
        mx, mn, avg = data.max(0), data.min(0), data.mean(0)
        feats = (data[:, :-1] - avg[:-1]) / (mx[:-1] - mn[:-1])
        n = int(len(data) * 0.8)
        sl = slice(0, n) if self.mode == 'train' else slice(n, None)
        self.x, self.y = feats[sl], data[sl, -1:]

    def __getitem__(self, i):
        return self.x[i], self.y[i]

    def __len__(self):
        return len(self.x)
