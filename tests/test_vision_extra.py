"""vision transforms / ops / datasets."""
import gzip
import os
import struct

import pytest

import numpy as np
import torch
from PIL import Image

import paddle
import paddle.vision.transforms as T
from paddle.vision import ops


def test_transforms_types_and_shapes():
    img = Image.fromarray((np.random.rand(32, 48, 3) * 255).astype('uint8'))
    x = T.Compose([T.RandomResizedCrop(24), T.RandomHorizontalFlip(), T.ColorJitter(0.4, 0.4, 0.4, 0.1),
                   T.ToTensor(), T.Normalize([0.5] * 3, [0.5] * 3)])(img)
    assert x.shape == [3, 24, 24]
    a = (np.random.rand(32, 48, 3) * 255).astype('uint8')
    assert T.Resize((16, 20))(a).shape == (16, 20, 3)
    assert T.Pad(2)(a).shape == (36, 52, 3)
    np.testing.assert_array_equal(T.functional.hflip(a), a[:, ::-1])
    np.testing.assert_array_equal(T.CenterCrop(10)(a), a[11:21, 19:29])
    t = paddle.to_tensor(np.random.rand(3, 32, 48).astype('float32'))
    assert T.RandomRotation(30)(t).shape == [3, 32, 48]
    assert T.functional.rotate(t, 90, expand=True).shape == [3, 48, 32]
    # identity affine is exact
    np.testing.assert_allclose(T.functional.affine(t, 0, (0, 0), 1.0, 0).numpy(), t.numpy(), atol=1e-6)
    g = T.functional.to_grayscale(img)
    assert g.mode == 'L'


def test_nms_and_roi_align():
    boxes = paddle.to_tensor([[0, 0, 10, 10], [1, 1, 11, 11], [20, 20, 30, 30], [0, 0, 10, 9]], dtype='float32')
    scores = paddle.to_tensor([0.9, 0.8, 0.7, 0.95])
    keep = ops.nms(boxes, 0.5, scores)
    assert keep.numpy().tolist() == [3, 2]
    keep2 = ops.nms(boxes, 0.5, scores, paddle.to_tensor([0, 1, 0, 0]), [0, 1])
    assert sorted(keep2.numpy().tolist()) == [1, 2, 3]
    feat = paddle.to_tensor(np.arange(2 * 1 * 8 * 8, dtype='float32').reshape(2, 1, 8, 8))
    rois = paddle.to_tensor([[0, 0, 4, 4], [2, 2, 6, 6]], dtype='float32')
    out = ops.roi_align(feat, rois, paddle.to_tensor([1, 1]), 2, sampling_ratio=2, aligned=False)
    assert out.shape == [2, 1, 2, 2]
    # bilinear mean over a linear ramp = value at the bin centre: x=1,y=1 → 9 in image 0
    assert abs(float(out.numpy()[0, 0, 0, 0]) - 9.0) < 1e-4
    rp = ops.roi_pool(feat, rois, paddle.to_tensor([1, 1]), 2)
    assert float(rp.numpy()[0, 0, 1, 1]) == 36.0


def test_deform_conv_zero_offset_equals_conv():
    x = paddle.randn([2, 4, 9, 9])
    w = paddle.randn([6, 4, 3, 3])
    off = paddle.zeros([2, 18, 9, 9])
    out = ops.deform_conv2d(x, off, w, padding=1)
    ref = torch.nn.functional.conv2d(x._t, w._t, padding=1)
    np.testing.assert_allclose(out.numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)
    layer = ops.DeformConv2D(4, 6, 3, padding=1)
    assert layer(x, off).shape == [2, 6, 9, 9]


def test_box_coder_roundtrip_and_prior_box():
    pb = paddle.to_tensor([[0.1, 0.1, 0.5, 0.5], [0.2, 0.3, 0.7, 0.9]])
    tb = paddle.to_tensor([[0.15, 0.12, 0.45, 0.55]])
    enc = ops.box_coder(pb, [0.1, 0.1, 0.2, 0.2], tb, 'encode_center_size')
    dec = ops.box_coder(pb, [0.1, 0.1, 0.2, 0.2], enc, 'decode_center_size')
    np.testing.assert_allclose(dec.numpy()[0, 0], tb.numpy()[0], atol=1e-5)
    b, v = ops.prior_box(paddle.zeros([1, 8, 4, 4]), paddle.zeros([1, 3, 32, 32]), [8.0], aspect_ratios=[2.0],
                         flip=True)
    assert b.shape == [4, 4, 3, 4] and v.shape == [4, 4, 3, 4]


def test_yolo_box_and_loss_shapes():
    x = paddle.randn([1, 3 * (5 + 4), 4, 4])
    boxes, scores = ops.yolo_box(x, paddle.to_tensor([[64, 64]]), [10, 13, 16, 30, 33, 23], 4, 0.01, 16)
    assert boxes.shape == [1, 48, 4] and scores.shape == [1, 48, 4]
    gt = paddle.to_tensor([[[0.5, 0.5, 0.3, 0.4]]])
    loss = ops.yolo_loss(x, gt, paddle.to_tensor([[1]]), [10, 13, 16, 30, 33, 23], [0, 1, 2], 4, 0.7, 16)
    assert loss.shape == [1] and float(loss) > 0


def test_mnist_and_folder(tmp_path):
    imgs = (np.random.rand(5, 28, 28) * 255).astype(np.uint8)
    with gzip.open(tmp_path / 'img.gz', 'wb') as f:
        f.write(struct.pack('>IIII', 2051, 5, 28, 28) + imgs.tobytes())
    with gzip.open(tmp_path / 'lab.gz', 'wb') as f:
        f.write(struct.pack('>II', 2049, 5) + bytes([1, 2, 3, 4, 5]))
    ds = paddle.vision.datasets.MNIST(str(tmp_path / 'img.gz'), str(tmp_path / 'lab.gz'), transform=T.ToTensor())
    x, y = ds[2]
    assert x.shape == [1, 28, 28] and int(y[0]) == 3
    for c in ('cat', 'dog'):
        os.makedirs(tmp_path / 'f' / c)
        Image.fromarray((np.random.rand(8, 8, 3) * 255).astype('uint8')).save(tmp_path / 'f' / c / 'a.png')
    fd = paddle.vision.datasets.DatasetFolder(str(tmp_path / 'f'))
    assert len(fd) == 2 and fd.classes == ['cat', 'dog']


@pytest.mark.parametrize('name', ['shufflenet_v2_x0_25', 'shufflenet_v2_x0_33', 'shufflenet_v2_x1_5',
                                  'shufflenet_v2_swish'])
def test_shufflenet_variants(name):
    """The four ShuffleNetV2 builders of reference vision/models/shufflenetv2.py:331-541."""
    import paddle
    from paddle.vision import models
    m = getattr(models, name)(num_classes=7)
    m.eval()
    assert m(paddle.randn([2, 3, 64, 64])).shape == [2, 7]
    last = {'shufflenet_v2_x0_25': 512, 'shufflenet_v2_x0_33': 512, 'shufflenet_v2_x1_5': 1024,
            'shufflenet_v2_swish': 1024}[name]
    assert m.fc.weight.shape == [last, 7]
