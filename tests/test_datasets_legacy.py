"""Text / vision corpora parsed from synthetic archives in the published layouts, the legacy
paddle.dataset reader creators, paddle.reader / paddle.batch, plus flags, regularizers, autotune
and the incubate LookAhead / ModelAverage optimizers."""
import gzip
import io
import os
import struct
import tarfile
import zipfile

import numpy as np
import pytest

import paddle


def _add(tf, name, data):
    ti = tarfile.TarInfo(name)
    ti.size = len(data)
    tf.addfile(ti, io.BytesIO(data))


def _imdb(path):
    with tarfile.open(path, 'w:gz') as tf:
        docs = {'train/pos/0.txt': b'a great movie, great fun!', 'train/pos/1.txt': b'great acting',
                'train/neg/0.txt': b'a bad movie.', 'test/pos/0.txt': b'great!', 'test/neg/0.txt': b'bad bad plot'}
        for k, v in docs.items():
            _add(tf, 'aclImdb/' + k, v)


def test_imdb(tmp_path):
    p = str(tmp_path / 'imdb.tar.gz')
    _imdb(p)
    tr = paddle.text.Imdb(p, 'train', cutoff=0)
    te = paddle.text.datasets.Imdb(p, 'test', cutoff=0)
    assert len(tr) == 3 and len(te) == 2
    w = tr.word_idx
    # tokens are bytes (as the reference's tokenizer), the most frequent word first, '<unk>' last
    assert w[b'great'] == 0 and w['<unk>'] == len(w) - 1
    doc, lab = tr[0]
    assert list(doc) == [w[b'a'], w[b'great'], w[b'movie'], w[b'great'], w[b'fun']] and lab.tolist() == [0]
    assert te[1][1].tolist() == [1]                       # neg label


def test_imikolov_ngram_and_seq(tmp_path):
    p = str(tmp_path / 'ptb.tgz')
    with tarfile.open(p, 'w:gz') as tf:
        _add(tf, './simple-examples/data/ptb.train.txt', b'the cat sat\nthe dog\n')
        _add(tf, './simple-examples/data/ptb.valid.txt', b'the cat\n')
        _add(tf, './simple-examples/data/ptb.test.txt', b'a cat ran\n')
    ng = paddle.text.Imikolov(p, 'NGRAM', window_size=3, mode='train', min_word_freq=0)
    w = ng.word_idx
    assert [tuple(x) for x in (ng[0], ng[1])] == [(w['<s>'], w['the'], w['cat']), (w['the'], w['cat'], w['sat'])]
    assert len(ng) == 3 + 2
    sq = paddle.text.Imikolov(p, 'SEQ', mode='test', min_word_freq=0)
    src, trg = sq[0]
    unk = w['<unk>']
    assert src.tolist() == [w['<s>'], unk, w['cat'], unk] and trg.tolist() == [unk, w['cat'], unk, w['<e>']]


def test_movielens(tmp_path):
    p = str(tmp_path / 'ml-1m.zip')
    with zipfile.ZipFile(p, 'w') as z:
        z.writestr('ml-1m/movies.dat', 'M1::Toy Story (1995)::Animation|Comedy\n2::Heat (1995)::Action\n'
                   .replace('M1', '1'))
        z.writestr('ml-1m/users.dat', '1::F::1::10::48067\n2::M::56::16::70072\n')
        z.writestr('ml-1m/ratings.dat', ''.join(f'{1 + i % 2}::{1 + i % 2}::{1 + i % 5}::97830{i}\n' for i in range(40)))
    tr = paddle.text.Movielens(p, 'train', test_ratio=0.25, rand_seed=3)
    te = paddle.text.Movielens(p, 'test', test_ratio=0.25, rand_seed=3)
    assert len(tr) + len(te) == 40 and len(te) > 0
    s = tr[0]
    uid = int(s[0][0])
    assert s[1].tolist() == [1 if uid == 1 else 0] and s[2].tolist() == [0 if uid == 1 else 6]
    assert float(s[-1][0]) in {2 * r - 5.0 for r in range(1, 6)}


def test_conll05(tmp_path):
    words = b'The\ncat\nsat\n.\n\n'
    props = b'-  (A0*\n-  *)\nsit  (V*)\n-  *\n\n'
    p = str(tmp_path / 'conll.tar.gz')
    with tarfile.open(p, 'w:gz') as tf:
        _add(tf, 'conll05st-release/test.wsj/words/test.wsj.words.gz', gzip.compress(words))
        _add(tf, 'conll05st-release/test.wsj/props/test.wsj.props.gz', gzip.compress(props))
    for name, txt in (('w', 'The\ncat\nsat\n.\nbos\neos\n'), ('v', 'sit\n'), ('t', 'B-A0\nI-A0\nB-V\nI-V\nO\n')):
        (tmp_path / name).write_text(txt)
    ds = paddle.text.Conll05st(p, str(tmp_path / 'w'), str(tmp_path / 'v'), str(tmp_path / 't'), emb_file='e')
    assert len(ds) == 1
    out = ds[0]
    assert out[0].tolist() == [0, 1, 2, 3]
    assert out[7].tolist() == [1, 1, 1, 1]                  # mark: predicate at 2, context +-2
    lab = ds.label_dict
    assert out[8].tolist() == [lab['B-A0'], lab['I-A0'], lab['B-V'], lab['O']]
    assert out[6].tolist() == [0] * 4                       # predicate id of 'sit'


def test_wmt14_and_wmt16(tmp_path):
    p14 = str(tmp_path / 'wmt14.tgz')
    with tarfile.open(p14, 'w:gz') as tf:
        _add(tf, 'wmt/src.dict', b'<s>\n<e>\n<unk>\nhello\nworld\n')
        _add(tf, 'wmt/trg.dict', b'<s>\n<e>\n<unk>\nbonjour\nmonde\n')
        _add(tf, 'wmt/train/train', b'hello world\tbonjour monde\nhello\tbonjour\nbad line\n')
    ds = paddle.text.WMT14(p14, 'train', dict_size=5)
    assert len(ds) == 2
    s, t, tn = ds[0]
    assert s.tolist() == [0, 3, 4, 1] and t.tolist() == [0, 3, 4] and tn.tolist() == [3, 4, 1]
    p16 = str(tmp_path / 'wmt16.tar.gz')
    with tarfile.open(p16, 'w:gz') as tf:
        _add(tf, 'wmt16/train', b'a b a\tx y\nb\tx\n')
        _add(tf, 'wmt16/test', b'a c\tz y\n')
    d16 = paddle.text.WMT16(p16, 'test', src_dict_size=10, trg_dict_size=10, lang='en',
                            dict_dir=str(tmp_path / 'dicts'))
    assert d16.src_dict['<s>'] == 0 and d16.src_dict['a'] == 3
    s, t, tn = d16[0]
    assert s.tolist() == [0, d16.src_dict['a'], 2, 1] and t.tolist()[0] == 0 and tn.tolist()[-1] == 1
    assert d16.get_dict('de', reverse=True)[0] == '<s>'


def _png(arr, mode=None):
    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(arr, mode).save(b, format='PNG')
    return b.getvalue()


def test_flowers_and_voc2012(tmp_path):
    import scipy.io as scio
    p = str(tmp_path / '102flowers.tgz')
    with tarfile.open(p, 'w:gz') as tf:
        for i in (1, 2, 3):
            from PIL import Image
            b = io.BytesIO()
            Image.fromarray(np.full((8, 8, 3), i * 40, np.uint8)).save(b, format='JPEG')
            _add(tf, 'jpg/image_%05d.jpg' % i, b.getvalue())
    scio.savemat(str(tmp_path / 'labels.mat'), {'labels': np.array([[5, 6, 7]])})
    scio.savemat(str(tmp_path / 'setid.mat'), {'tstid': np.array([[1, 3]]), 'trnid': np.array([[2]]),
                                               'valid': np.array([[3]])})
    fl = paddle.vision.datasets.Flowers(p, str(tmp_path / 'labels.mat'), str(tmp_path / 'setid.mat'), mode='train',
                                        backend='cv2')
    assert len(fl) == 2
    img, lab = fl[1]
    assert img.shape == (8, 8, 3) and lab.tolist() == [7]
    vp = str(tmp_path / 'voc.tar')
    with tarfile.open(vp, 'w') as tf:
        _add(tf, 'VOCdevkit/VOC2012/ImageSets/Segmentation/val.txt', b'x1\n')
        _add(tf, 'VOCdevkit/VOC2012/JPEGImages/x1.jpg', _png(np.zeros((4, 5, 3), np.uint8)))
        _add(tf, 'VOCdevkit/VOC2012/SegmentationClass/x1.png', _png(np.eye(4, 5, dtype=np.uint8), 'L'))
    voc = paddle.vision.datasets.VOC2012(vp, mode='valid', backend='cv2')
    img, lab = voc[0]
    assert len(voc) == 1 and img.shape == (4, 5, 3) and lab.tolist() == np.eye(4, 5).tolist()


def _idx(path, arr, magic):
    with gzip.open(path, 'wb') as f:
        f.write(struct.pack('>I', magic) + b''.join(struct.pack('>I', d) for d in arr.shape) + arr.tobytes())


def test_legacy_dataset_readers(tmp_path, monkeypatch):
    home = tmp_path / 'home'
    monkeypatch.setattr(paddle.dataset.common, 'DATA_HOME', str(home))
    (home / 'mnist').mkdir(parents=True)
    imgs = np.arange(3 * 28 * 28, dtype=np.uint32).reshape(3, 28, 28).astype(np.uint8)
    _idx(home / 'mnist' / 'train-images-idx3-ubyte.gz', imgs, 2051)
    _idx(home / 'mnist' / 'train-labels-idx1-ubyte.gz', np.array([4, 1, 9], np.uint8), 2049)
    samples = list(paddle.dataset.mnist.train()())
    assert len(samples) == 3 and samples[2][1] == 9
    np.testing.assert_allclose(samples[0][0], imgs[0].reshape(-1) / 255.0 * 2 - 1, rtol=1e-6, atol=1e-6)
    (home / 'uci_housing').mkdir()
    np.savetxt(home / 'uci_housing' / 'housing.data', np.random.RandomState(0).rand(10, 14))
    assert len(list(paddle.dataset.uci_housing.train()())) == 8
    (home / 'cifar').mkdir()
    rec = np.zeros((2, 3073), np.uint8)
    rec[:, 0] = [3, 7]
    rec[1, 1:] = 255
    with tarfile.open(home / 'cifar' / 'cifar-10-binary.tar.gz', 'w:gz') as tf:
        _add(tf, 'cifar-10-batches-bin/data_batch_1.bin', rec.tobytes())
    cs = list(paddle.dataset.cifar.train10()())
    assert [c[1] for c in cs] == [3, 7] and cs[1][0].max() == 1.0 and cs[0][0].shape == (3072,)
    (home / 'imdb').mkdir()
    _imdb(str(home / 'imdb' / 'aclImdb_v1.tar.gz'))
    wd = paddle.dataset.imdb.word_dict(cutoff=0)
    assert len(list(paddle.dataset.imdb.train(wd)())) == 3
    with pytest.raises(RuntimeError):
        list(paddle.dataset.wmt14.train(10)())  # archive absent: no download
    # legacy decorators + paddle.batch
    r = paddle.reader.shuffle(paddle.dataset.uci_housing.train(), buf_size=4)
    batches = list(paddle.batch(r, batch_size=3)())
    assert [len(b) for b in batches] == [3, 3, 2]
    assert len(list(paddle.reader.firstn(r, 5)())) == 5
    img = paddle.dataset.image.simple_transform(np.zeros((40, 60, 3), np.uint8), 32, 24, False, mean=[1, 2, 3])
    assert img.shape == (3, 24, 24) and img[0, 0, 0] == -1


def test_flags_roundtrip():
    old = paddle.get_flags(['FLAGS_check_nan_inf'])['FLAGS_check_nan_inf']
    paddle.set_flags({'FLAGS_check_nan_inf': True})
    try:
        assert paddle.get_flags('FLAGS_check_nan_inf')['FLAGS_check_nan_inf'] is True
    finally:
        paddle.set_flags({'FLAGS_check_nan_inf': old})
    with pytest.raises(Exception):
        paddle.set_flags({'FLAGS_not_a_real_flag_xyz': 1})


@pytest.mark.parametrize('reg', ['l1', 'l2'])
def test_regularizers_match_formula(reg):
    paddle.seed(1)
    lin = paddle.nn.Linear(4, 3)
    w0 = lin.weight.numpy().copy()
    coeff = 0.1
    r = paddle.regularizer.L1Decay(coeff) if reg == 'l1' else paddle.regularizer.L2Decay(coeff)
    opt = paddle.optimizer.SGD(learning_rate=0.5, parameters=lin.parameters(), weight_decay=r)
    x = paddle.randn([5, 4])
    lin(x).sum().backward()
    g = lin.weight.grad.numpy().copy()
    opt.step()
    extra = coeff * (np.sign(w0) if reg == 'l1' else w0)
    np.testing.assert_allclose(lin.weight.numpy(), w0 - 0.5 * (g + extra), rtol=1e-5, atol=1e-6)


def test_autotune_config():
    paddle.incubate.autotune.set_config({'kernel': {'enable': True, 'tuning_range': [1, 3]}})
    cfg = paddle.incubate.autotune.get_config() if hasattr(paddle.incubate.autotune, 'get_config') else None
    assert cfg is None or cfg['kernel']['enable'] is True


def test_lookahead_and_model_average():
    paddle.seed(0)
    lin = paddle.nn.Linear(3, 1)
    w0 = lin.weight.numpy().copy()
    inner = paddle.optimizer.SGD(learning_rate=0.1, parameters=lin.parameters())
    la = paddle.incubate.LookAhead(inner, alpha=0.5, k=2)
    x = paddle.ones([4, 3])
    fast = []
    for _ in range(2):
        lin(x).sum().backward()
        la.step()
        la.clear_grad()
        fast.append(lin.weight.numpy().copy())
    # the slow weights start from the parameters after the first step (reference lookahead.py:262);
    # every k steps slow <- slow + alpha (fast - slow) and fast <- slow
    g = 4.0  # d(sum(x @ w))/dw = 4 for every weight
    slow = w0 - 0.1 * g
    fast_k = w0 - 2 * 0.1 * g
    np.testing.assert_allclose(fast[-1], slow + 0.5 * (fast_k - slow), rtol=1e-5)
    lin2 = paddle.nn.Linear(3, 1)
    opt = paddle.optimizer.SGD(learning_rate=0.1, parameters=lin2.parameters())
    ma = paddle.incubate.ModelAverage(0.15, parameters=lin2.parameters(), min_average_window=2,
                                      max_average_window=10)
    ws = []
    for _ in range(3):
        lin2(x).sum().backward()
        opt.step()
        ma.step()
        opt.clear_grad()
        ws.append(lin2.weight.numpy().copy())
    with ma.apply():
        avg = lin2.weight.numpy().copy()
    np.testing.assert_allclose(lin2.weight.numpy(), ws[-1], rtol=1e-6)   # restored after apply()
    assert np.all(avg >= np.min(ws, 0) - 1e-6) and np.all(avg <= np.max(ws, 0) + 1e-6)
