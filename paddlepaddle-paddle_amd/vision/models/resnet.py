"""ResNet / ResNeXt / Wide-ResNet (reference: python/paddle/vision/models/resnet.py).

Same sublayer names as the reference (conv1/bn1/layer1..4/fc, blocks conv1..3/bn1..3/downsample)
so reference checkpoints map 1:1.  Both data formats run the channels-last HIP kernels: NHWC
directly, NCHW as NCHW views with channels-last strides (nn/functional/conv.py).
"""
from contextlib import nullcontext as _nullctx

import torch

from ... import nn
from ... import ops
from ...core.tensor import _wrap, _unwrap


RESIDUAL_GRAD_SINK = True  # identity blocks: conv1's dgrad GEMM accumulates the residual gradient


def _nhwc(bn, t):
    """The channels-last image of an activation: itself for NHWC layers, the NHWC view of an
    NCHW tensor with channels-last strides (what a routed NCHW conv2d returns), else None."""
    if bn._data_format[-1] == 'C':
        return t
    if t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last):
        return t.permute(0, 2, 3, 1)
    return None


def _fused_bn_ok(bn, t):
    if not (bn.training and isinstance(bn, nn.BatchNorm2D) and bn._use_global_stats is not True and ops.use_hip(t)):
        return False
    tn = _nhwc(bn, t)
    return tn is not None and ops.batchnorm.supported(tn, None if bn.weight is None else bn.weight._t)


def _bn_act(bn, x, relu=True, residual=None, dz_sink=None):
    """act(bn(x) [+ residual]) — one csrc/batchnorm.hip pass each way for channels-last training
    on the GPU (fused_bn_add_activation); the plain layer sequence otherwise.  NCHW layers run the
    same kernels on the channels-last image (ops.conv returns NCHW views with NHWC strides)."""
    t = _unwrap(x)
    if _fused_bn_ok(bn, t):
        r = None
        if residual is not None:
            r = _nhwc(bn, _unwrap(residual))
            if r is None:  # an NCHW-contiguous residual: repack it once
                r = _unwrap(residual).permute(0, 2, 3, 1).contiguous()
        y = ops.batchnorm.bn_act_nhwc(
            _nhwc(bn, t), None if bn.weight is None else bn.weight._t, None if bn.bias is None else bn.bias._t,
            bn._mean._t, bn._variance._t, bn._epsilon, bn._momentum, True, relu, r, dz_sink)
        return _wrap(y if bn._data_format[-1] == 'C' else y.permute(0, 3, 1, 2))
    y = bn(x)
    if residual is not None:
        y = y + residual
    return nn.functional.relu(y) if relu else y


class BasicBlock(nn.Layer):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64, dilation=1,
                 norm_layer=None, data_format='NCHW'):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2D
        self.conv1 = nn.Conv2D(inplanes, planes, 3, padding=1, stride=stride, bias_attr=False, data_format=data_format)
        self.bn1 = norm_layer(planes, data_format=data_format)
        self.relu = nn.ReLU()
        self.conv2 = nn.Conv2D(planes, planes, 3, padding=1, bias_attr=False, data_format=data_format)
        self.bn2 = norm_layer(planes, data_format=data_format)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        out = _bn_act(self.bn1, self.conv1(x))
        out = self.conv2(out)
        if self.downsample is not None:
            identity = self.downsample(x)
        return _bn_act(self.bn2, out, True, identity)


class BottleneckBlock(nn.Layer):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64, dilation=1,
                 norm_layer=None, data_format='NCHW'):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2D
        width = int(planes * (base_width / 64.0)) * groups
        df = data_format
        self.conv1 = nn.Conv2D(inplanes, width, 1, bias_attr=False, data_format=df)
        self.bn1 = norm_layer(width, data_format=df)
        self.conv2 = nn.Conv2D(width, width, 3, padding=dilation, stride=stride, groups=groups, dilation=dilation,
                               bias_attr=False, data_format=df)
        self.bn2 = norm_layer(width, data_format=df)
        self.conv3 = nn.Conv2D(width, planes * self.expansion, 1, bias_attr=False, data_format=df)
        self.bn3 = norm_layer(planes * self.expansion, data_format=df)
        self.relu = nn.ReLU()
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        # identity block: the residual gradient is accumulated by conv1's data-gradient GEMM
        # (ops.conv.GradSink) instead of a separate autograd add of the two branch gradients
        sink = ops.conv.GradSink() if (RESIDUAL_GRAD_SINK and self.downsample is None
                                       and _fused_bn_ok(self.bn3, _unwrap(x))) else None
        xk = _nhwc(self.bn3, _unwrap(x))  # the tensor conv2d_nhwc sees (shared-dgrad key)
        # downsample block: conv1 and the shortcut conv read the same x; their data gradients meet
        # in one tensor (ops.conv.SharedDgrad) instead of an autograd add
        shared = ops.conv.SharedDgrad() if (RESIDUAL_GRAD_SINK and self.downsample is not None
                                            and _fused_bn_ok(self.bn3, _unwrap(x))) else None
        if sink is not None:
            with ops.conv.dgrad_sink(sink):
                out = self.conv1(x)
        elif shared is not None:
            with ops.conv.shared_dgrad(xk, shared):
                out = self.conv1(x)
        else:
            out = self.conv1(x)
        out = _bn_act(self.bn1, out)
        out = _bn_act(self.bn2, self.conv2(out))
        out = self.conv3(out)
        if self.downsample is not None:
            if shared is not None:
                with ops.conv.shared_dgrad(xk, shared):
                    identity = self.downsample(x)
            else:
                identity = self.downsample(x)
        return _bn_act(self.bn3, out, True, identity, dz_sink=sink if sink is not None and sink.armed else None)


class ResNet(nn.Layer):
    def __init__(self, block, depth=50, width=64, num_classes=1000, with_pool=True, groups=1, data_format='NCHW'):
        super().__init__()
        layer_cfg = {18: [2, 2, 2, 2], 34: [3, 4, 6, 3], 50: [3, 4, 6, 3], 101: [3, 4, 23, 3], 152: [3, 8, 36, 3]}
        layers = layer_cfg[depth]
        self.groups, self.base_width = groups, width
        self.num_classes, self.with_pool = num_classes, with_pool
        self.data_format = data_format
        self._norm_layer = nn.BatchNorm2D
        self.inplanes = 64
        self.dilation = 1
        self.conv1 = nn.Conv2D(3, self.inplanes, 7, stride=2, padding=3, bias_attr=False, data_format=data_format)
        self.bn1 = self._norm_layer(self.inplanes, data_format=data_format)
        self.relu = nn.ReLU()
        self.maxpool = nn.MaxPool2D(3, stride=2, padding=1, data_format=data_format)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        if with_pool:
            self.avgpool = nn.AdaptiveAvgPool2D((1, 1), data_format=data_format)
        if num_classes > 0:
            self.fc = nn.Linear(512 * block.expansion, num_classes)

    def _make_layer(self, block, planes, blocks, stride=1, dilate=False):
        df = self.data_format
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                nn.Conv2D(self.inplanes, planes * block.expansion, 1, stride=stride, bias_attr=False, data_format=df),
                self._norm_layer(planes * block.expansion, data_format=df))
        layers = [block(self.inplanes, planes, stride, downsample, self.groups, self.base_width, 1, None, df)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, groups=self.groups, base_width=self.base_width,
                                data_format=df))
        return nn.Sequential(*layers)

    def forward(self, x):
        # every convolution here feeds a batch norm: in training, the conv epilogues also emit the
        # norm's batch statistics (ops.conv.fused_bn_stats), so the norms skip their statistics pass
        with ops.conv.fused_bn_stats() if self.training else _nullctx():
            # stem: conv -> BN + ReLU in one fused pass each way (a separate ReLU cost a clamp over the
            # 256x112x112x64 activation forward and a threshold pass backward, 0.35 ms per step)
            x = self.maxpool(_bn_act(self.bn1, self.conv1(x)))
            x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        if self.with_pool:
            x = self.avgpool(x)
        if self.num_classes > 0:
            x = x.flatten(1)
            x = self.fc(x)
        return x


def _resnet(arch, Block, depth, pretrained, **kwargs):
    if pretrained:
        raise ValueError("pretrained weights are not available offline")
    return ResNet(Block, depth, **kwargs)


def resnet18(pretrained=False, **kw):
    return _resnet('resnet18', BasicBlock, 18, pretrained, **kw)


def resnet34(pretrained=False, **kw):
    return _resnet('resnet34', BasicBlock, 34, pretrained, **kw)


def resnet50(pretrained=False, **kw):
    return _resnet('resnet50', BottleneckBlock, 50, pretrained, **kw)


def resnet101(pretrained=False, **kw):
    return _resnet('resnet101', BottleneckBlock, 101, pretrained, **kw)


def resnet152(pretrained=False, **kw):
    return _resnet('resnet152', BottleneckBlock, 152, pretrained, **kw)


def resnext50_32x4d(pretrained=False, **kw):
    return _resnet('resnext50_32x4d', BottleneckBlock, 50, pretrained, groups=32, width=4, **kw)


def resnext50_64x4d(pretrained=False, **kw):
    return _resnet('resnext50_64x4d', BottleneckBlock, 50, pretrained, groups=64, width=4, **kw)


def resnext101_32x4d(pretrained=False, **kw):
    return _resnet('resnext101_32x4d', BottleneckBlock, 101, pretrained, groups=32, width=4, **kw)


def resnext101_64x4d(pretrained=False, **kw):
    return _resnet('resnext101_64x4d', BottleneckBlock, 101, pretrained, groups=64, width=4, **kw)


def resnext152_32x4d(pretrained=False, **kw):
    return _resnet('resnext152_32x4d', BottleneckBlock, 152, pretrained, groups=32, width=4, **kw)


def resnext152_64x4d(pretrained=False, **kw):
    return _resnet('resnext152_64x4d', BottleneckBlock, 152, pretrained, groups=64, width=4, **kw)


def wide_resnet50_2(pretrained=False, **kw):
    return _resnet('wide_resnet50_2', BottleneckBlock, 50, pretrained, width=128, **kw)


def wide_resnet101_2(pretrained=False, **kw):
    return _resnet('wide_resnet101_2', BottleneckBlock, 101, pretrained, width=128, **kw)
