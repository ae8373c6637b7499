"""Classic CNN zoo (reference: python/paddle/vision/models/{vgg,alexnet,mobilenetv1,mobilenetv2,mobilenetv3,
squeezenet,shufflenetv2,densenet,googlenet,inceptionv3}.py).  Architectures follow the reference
definitions; ``pretrained=True`` is unavailable offline."""
from ... import nn
from ...nn import functional as F
from ...tensor.manipulation import concat, reshape, transpose, flatten


def _no_pretrained(p):
    if p:
        raise ValueError("pretrained weights are not available offline")


# ----------------------------------------------------------------------------- VGG
class VGG(nn.Layer):
    def __init__(self, features, num_classes=1000, with_pool=True):
        super().__init__()
        self.features = features
        self.num_classes, self.with_pool = num_classes, with_pool
        if with_pool:
            self.avgpool = nn.AdaptiveAvgPool2D((7, 7))
        if num_classes > 0:
            self.classifier = nn.Sequential(nn.Linear(512 * 7 * 7, 4096), nn.ReLU(), nn.Dropout(),
                                            nn.Linear(4096, 4096), nn.ReLU(), nn.Dropout(),
                                            nn.Linear(4096, num_classes))

    def forward(self, x):
        x = self.features(x)
        if self.with_pool:
            x = self.avgpool(x)
        if self.num_classes > 0:
            x = self.classifier(flatten(x, 1))
        return x


_VGG_CFG = {'A': [64, 'M', 128, 'M', 256, 256, 'M', 512, 512, 'M', 512, 512, 'M'],
            'B': [64, 64, 'M', 128, 128, 'M', 256, 256, 'M', 512, 512, 'M', 512, 512, 'M'],
            'D': [64, 64, 'M', 128, 128, 'M', 256, 256, 256, 'M', 512, 512, 512, 'M', 512, 512, 512, 'M'],
            'E': [64, 64, 'M', 128, 128, 'M', 256, 256, 256, 256, 'M', 512, 512, 512, 512, 'M', 512, 512, 512, 512,
                  'M']}


def _vgg_features(cfg, batch_norm):
    layers, c = [], 3
    for v in cfg:
        if v == 'M':
            layers.append(nn.MaxPool2D(2, 2))
        else:
            layers.append(nn.Conv2D(c, v, 3, padding=1))
            if batch_norm:
                layers.append(nn.BatchNorm2D(v))
            layers.append(nn.ReLU())
            c = v
    return nn.Sequential(*layers)


def vgg11(pretrained=False, batch_norm=False, **kw):
    _no_pretrained(pretrained)
    return VGG(_vgg_features(_VGG_CFG['A'], batch_norm), **kw)


def vgg13(pretrained=False, batch_norm=False, **kw):
    _no_pretrained(pretrained)
    return VGG(_vgg_features(_VGG_CFG['B'], batch_norm), **kw)


def vgg16(pretrained=False, batch_norm=False, **kw):
    _no_pretrained(pretrained)
    return VGG(_vgg_features(_VGG_CFG['D'], batch_norm), **kw)


def vgg19(pretrained=False, batch_norm=False, **kw):
    _no_pretrained(pretrained)
    return VGG(_vgg_features(_VGG_CFG['E'], batch_norm), **kw)


# ----------------------------------------------------------------------------- AlexNet
class AlexNet(nn.Layer):
    def __init__(self, num_classes=1000):
        super().__init__()
        self.num_classes = num_classes
        self.features = nn.Sequential(
            nn.Conv2D(3, 64, 11, stride=4, padding=2), nn.ReLU(), nn.MaxPool2D(3, 2),
            nn.Conv2D(64, 192, 5, padding=2), nn.ReLU(), nn.MaxPool2D(3, 2),
            nn.Conv2D(192, 384, 3, padding=1), nn.ReLU(),
            nn.Conv2D(384, 256, 3, padding=1), nn.ReLU(),
            nn.Conv2D(256, 256, 3, padding=1), nn.ReLU(), nn.MaxPool2D(3, 2))
        self.avgpool = nn.AdaptiveAvgPool2D((6, 6))
        if num_classes > 0:
            self.classifier = nn.Sequential(nn.Dropout(), nn.Linear(256 * 36, 4096), nn.ReLU(), nn.Dropout(),
                                            nn.Linear(4096, 4096), nn.ReLU(), nn.Linear(4096, num_classes))

    def forward(self, x):
        x = self.avgpool(self.features(x))
        return self.classifier(flatten(x, 1)) if self.num_classes > 0 else x


def alexnet(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return AlexNet(**kw)


# ----------------------------------------------------------------------------- MobileNets
def _make_divisible(v, divisor=8, min_value=None):
    min_value = min_value or divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


class ConvBNLayer(nn.Layer):
    def __init__(self, cin, cout, k, stride=1, padding=0, groups=1, act='relu'):
        super().__init__()
        self.conv = nn.Conv2D(cin, cout, k, stride=stride, padding=padding, groups=groups, bias_attr=False)
        self.bn = nn.BatchNorm2D(cout)
        self.act = {'relu': nn.ReLU(), 'relu6': nn.ReLU6(), 'hardswish': nn.Hardswish(), 'swish': nn.Swish(),
                    None: None}[act]

    def forward(self, x):
        x = self.bn(self.conv(x))
        return self.act(x) if self.act is not None else x


class MobileNetV1(nn.Layer):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__()
        s = lambda c: int(c * scale)  # noqa: E731
        cfg = [(32, 64, 1), (64, 128, 2), (128, 128, 1), (128, 256, 2), (256, 256, 1), (256, 512, 2)] + \
              [(512, 512, 1)] * 5 + [(512, 1024, 2), (1024, 1024, 1)]
        layers = [ConvBNLayer(3, s(32), 3, 2, 1)]
        for cin, cout, st in cfg:
            layers += [ConvBNLayer(s(cin), s(cin), 3, st, 1, groups=s(cin)), ConvBNLayer(s(cin), s(cout), 1)]
        self.features = nn.Sequential(*layers)
        self.num_classes, self.with_pool = num_classes, with_pool
        if with_pool:
            self.pool2d_avg = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.fc = nn.Linear(s(1024), num_classes)

    def forward(self, x):
        x = self.features(x)
        if self.with_pool:
            x = self.pool2d_avg(x)
        return self.fc(flatten(x, 1)) if self.num_classes > 0 else x


class InvertedResidual(nn.Layer):
    def __init__(self, inp, oup, stride, expand_ratio):
        super().__init__()
        hidden = int(round(inp * expand_ratio))
        self.use_res_connect = stride == 1 and inp == oup
        layers = []
        if expand_ratio != 1:
            layers.append(ConvBNLayer(inp, hidden, 1, act='relu6'))
        layers += [ConvBNLayer(hidden, hidden, 3, stride, 1, groups=hidden, act='relu6'),
                   ConvBNLayer(hidden, oup, 1, act=None)]
        self.conv = nn.Sequential(*layers)

    def forward(self, x):
        return x + self.conv(x) if self.use_res_connect else self.conv(x)


class MobileNetV2(nn.Layer):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__()
        cfg = [[1, 16, 1, 1], [6, 24, 2, 2], [6, 32, 3, 2], [6, 64, 4, 2], [6, 96, 3, 1], [6, 160, 3, 2],
               [6, 320, 1, 1]]
        inp = _make_divisible(32 * scale)
        self.last_channel = _make_divisible(1280 * max(1.0, scale))
        features = [ConvBNLayer(3, inp, 3, 2, 1, act='relu6')]
        for t, c, n, s in cfg:
            out = _make_divisible(c * scale)
            for i in range(n):
                features.append(InvertedResidual(inp, out, s if i == 0 else 1, t))
                inp = out
        features.append(ConvBNLayer(inp, self.last_channel, 1, act='relu6'))
        self.features = nn.Sequential(*features)
        self.num_classes, self.with_pool = num_classes, with_pool
        if with_pool:
            self.pool2d_avg = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.classifier = nn.Sequential(nn.Dropout(0.2), nn.Linear(self.last_channel, num_classes))

    def forward(self, x):
        x = self.features(x)
        if self.with_pool:
            x = self.pool2d_avg(x)
        return self.classifier(flatten(x, 1)) if self.num_classes > 0 else x


class SqueezeExcitation(nn.Layer):
    def __init__(self, c, squeeze):
        super().__init__()
        self.avgpool = nn.AdaptiveAvgPool2D(1)
        self.fc1 = nn.Conv2D(c, squeeze, 1)
        self.relu = nn.ReLU()
        self.fc2 = nn.Conv2D(squeeze, c, 1)
        self.hardsigmoid = nn.Hardsigmoid(slope=0.2, offset=0.5)

    def forward(self, x):
        s = self.hardsigmoid(self.fc2(self.relu(self.fc1(self.avgpool(x)))))
        return x * s


class _MBV3Block(nn.Layer):
    def __init__(self, cin, k, exp, cout, use_se, act, stride):
        super().__init__()
        self.use_res = stride == 1 and cin == cout
        layers = []
        if exp != cin:
            layers.append(ConvBNLayer(cin, exp, 1, act=act))
        layers.append(ConvBNLayer(exp, exp, k, stride, (k - 1) // 2, groups=exp, act=act))
        if use_se:
            layers.append(SqueezeExcitation(exp, _make_divisible(exp // 4)))
        layers.append(ConvBNLayer(exp, cout, 1, act=None))
        self.block = nn.Sequential(*layers)

    def forward(self, x):
        y = self.block(x)
        return x + y if self.use_res else y


class MobileNetV3(nn.Layer):
    def __init__(self, config, last_channel, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__()
        inp = _make_divisible(16 * scale)
        layers = [ConvBNLayer(3, inp, 3, 2, 1, act='hardswish')]
        for k, exp, c, se, act, s in config:
            out = _make_divisible(c * scale)
            layers.append(_MBV3Block(inp, k, _make_divisible(exp * scale), out, se, act, s))
            inp = out
        last_conv = 6 * inp
        layers.append(ConvBNLayer(inp, last_conv, 1, act='hardswish'))
        self.features = nn.Sequential(*layers)
        self.num_classes, self.with_pool = num_classes, with_pool
        if with_pool:
            self.avgpool = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.classifier = nn.Sequential(nn.Linear(last_conv, last_channel), nn.Hardswish(), nn.Dropout(0.2),
                                            nn.Linear(last_channel, num_classes))

    def forward(self, x):
        x = self.features(x)
        if self.with_pool:
            x = self.avgpool(x)
        return self.classifier(flatten(x, 1)) if self.num_classes > 0 else x


class MobileNetV3Small(MobileNetV3):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        cfg = [(3, 16, 16, True, 'relu', 2), (3, 72, 24, False, 'relu', 2), (3, 88, 24, False, 'relu', 1),
               (5, 96, 40, True, 'hardswish', 2), (5, 240, 40, True, 'hardswish', 1),
               (5, 240, 40, True, 'hardswish', 1), (5, 120, 48, True, 'hardswish', 1),
               (5, 144, 48, True, 'hardswish', 1), (5, 288, 96, True, 'hardswish', 2),
               (5, 576, 96, True, 'hardswish', 1), (5, 576, 96, True, 'hardswish', 1)]
        super().__init__(cfg, _make_divisible(1024 * scale), scale, num_classes, with_pool)


class MobileNetV3Large(MobileNetV3):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        cfg = [(3, 16, 16, False, 'relu', 1), (3, 64, 24, False, 'relu', 2), (3, 72, 24, False, 'relu', 1),
               (5, 72, 40, True, 'relu', 2), (5, 120, 40, True, 'relu', 1), (5, 120, 40, True, 'relu', 1),
               (3, 240, 80, False, 'hardswish', 2), (3, 200, 80, False, 'hardswish', 1),
               (3, 184, 80, False, 'hardswish', 1), (3, 184, 80, False, 'hardswish', 1),
               (3, 480, 112, True, 'hardswish', 1), (3, 672, 112, True, 'hardswish', 1),
               (5, 672, 160, True, 'hardswish', 2), (5, 960, 160, True, 'hardswish', 1),
               (5, 960, 160, True, 'hardswish', 1)]
        super().__init__(cfg, _make_divisible(1280 * scale), scale, num_classes, with_pool)


def mobilenet_v1(pretrained=False, scale=1.0, **kw):
    _no_pretrained(pretrained)
    return MobileNetV1(scale=scale, **kw)


def mobilenet_v2(pretrained=False, scale=1.0, **kw):
    _no_pretrained(pretrained)
    return MobileNetV2(scale=scale, **kw)


def mobilenet_v3_small(pretrained=False, scale=1.0, **kw):
    _no_pretrained(pretrained)
    return MobileNetV3Small(scale=scale, **kw)


def mobilenet_v3_large(pretrained=False, scale=1.0, **kw):
    _no_pretrained(pretrained)
    return MobileNetV3Large(scale=scale, **kw)


# ----------------------------------------------------------------------------- SqueezeNet
class _Fire(nn.Layer):
    def __init__(self, cin, sq, e1, e3):
        super().__init__()
        self.squeeze = nn.Conv2D(cin, sq, 1)
        self.expand1x1 = nn.Conv2D(sq, e1, 1)
        self.expand3x3 = nn.Conv2D(sq, e3, 3, padding=1)

    def forward(self, x):
        x = F.relu(self.squeeze(x))
        return concat([F.relu(self.expand1x1(x)), F.relu(self.expand3x3(x))], axis=1)


class SqueezeNet(nn.Layer):
    def __init__(self, version, num_classes=1000, with_pool=True):
        super().__init__()
        if version == '1.0':
            self.features = nn.Sequential(
                nn.Conv2D(3, 96, 7, stride=2), nn.ReLU(), nn.MaxPool2D(3, 2, ceil_mode=True),
                _Fire(96, 16, 64, 64), _Fire(128, 16, 64, 64), _Fire(128, 32, 128, 128),
                nn.MaxPool2D(3, 2, ceil_mode=True), _Fire(256, 32, 128, 128), _Fire(256, 48, 192, 192),
                _Fire(384, 48, 192, 192), _Fire(384, 64, 256, 256), nn.MaxPool2D(3, 2, ceil_mode=True),
                _Fire(512, 64, 256, 256))
        else:
            self.features = nn.Sequential(
                nn.Conv2D(3, 64, 3, stride=2), nn.ReLU(), nn.MaxPool2D(3, 2, ceil_mode=True),
                _Fire(64, 16, 64, 64), _Fire(128, 16, 64, 64), nn.MaxPool2D(3, 2, ceil_mode=True),
                _Fire(128, 32, 128, 128), _Fire(256, 32, 128, 128), nn.MaxPool2D(3, 2, ceil_mode=True),
                _Fire(256, 48, 192, 192), _Fire(384, 48, 192, 192), _Fire(384, 64, 256, 256),
                _Fire(512, 64, 256, 256))
        self.num_classes, self.with_pool = num_classes, with_pool
        if num_classes > 0:
            self._drop = nn.Dropout(0.5)
            self._conv = nn.Conv2D(512, num_classes, 1)
        self._avg_pool = nn.AdaptiveAvgPool2D(1)

    def forward(self, x):
        x = self.features(x)
        if self.num_classes > 0:
            x = F.relu(self._conv(self._drop(x)))
        if self.with_pool:
            x = self._avg_pool(x)
        return flatten(x, 1) if self.num_classes > 0 else x


def squeezenet1_0(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return SqueezeNet('1.0', **kw)


def squeezenet1_1(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return SqueezeNet('1.1', **kw)


# ----------------------------------------------------------------------------- ShuffleNetV2
def _channel_shuffle(x, groups):
    return F.channel_shuffle(x, groups)


class _ShuffleUnit(nn.Layer):
    def __init__(self, cin, cout, stride, act='relu'):
        super().__init__()
        self.stride = stride
        branch = cout // 2
        if stride > 1:
            self.branch1 = nn.Sequential(ConvBNLayer(cin, cin, 3, stride, 1, groups=cin, act=None),
                                         ConvBNLayer(cin, branch, 1, act=act))
        b2_in = cin if stride > 1 else branch
        self.branch2 = nn.Sequential(ConvBNLayer(b2_in, branch, 1, act=act),
                                     ConvBNLayer(branch, branch, 3, stride, 1, groups=branch, act=None),
                                     ConvBNLayer(branch, branch, 1, act=act))

    def forward(self, x):
        if self.stride == 1:
            x1, x2 = x.chunk(2, axis=1)
            out = concat([x1, self.branch2(x2)], axis=1)
        else:
            out = concat([self.branch1(x), self.branch2(x)], axis=1)
        return _channel_shuffle(out, 2)


class ShuffleNetV2(nn.Layer):
    def __init__(self, scale=1.0, act='relu', num_classes=1000, with_pool=True):
        super().__init__()
        chans = {0.25: [24, 24, 48, 96, 512], 0.33: [24, 32, 64, 128, 512], 0.5: [24, 48, 96, 192, 1024],
                 1.0: [24, 116, 232, 464, 1024], 1.5: [24, 176, 352, 704, 1024], 2.0: [24, 224, 488, 976, 2048]}[scale]
        self.conv1 = ConvBNLayer(3, chans[0], 3, 2, 1, act=act)
        self.max_pool = nn.MaxPool2D(3, 2, padding=1)
        blocks = []
        cin = chans[0]
        for stage, reps in enumerate([4, 8, 4]):
            cout = chans[stage + 1]
            for i in range(reps):
                blocks.append(_ShuffleUnit(cin, cout, 2 if i == 0 else 1, act))
                cin = cout
        self.blocks = nn.Sequential(*blocks)
        self.last_conv = ConvBNLayer(cin, chans[-1], 1, act=act)
        self.num_classes, self.with_pool = num_classes, with_pool
        if with_pool:
            self.pool2d_avg = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.fc = nn.Linear(chans[-1], num_classes)

    def forward(self, x):
        x = self.last_conv(self.blocks(self.max_pool(self.conv1(x))))
        if self.with_pool:
            x = self.pool2d_avg(x)
        return self.fc(flatten(x, 1)) if self.num_classes > 0 else x


def shufflenet_v2_x1_0(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return ShuffleNetV2(1.0, **kw)


def shufflenet_v2_x0_5(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return ShuffleNetV2(0.5, **kw)


def shufflenet_v2_x2_0(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return ShuffleNetV2(2.0, **kw)


def shufflenet_v2_x0_25(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return ShuffleNetV2(0.25, **kw)


def shufflenet_v2_x0_33(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return ShuffleNetV2(0.33, **kw)


def shufflenet_v2_x1_5(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return ShuffleNetV2(1.5, **kw)


def shufflenet_v2_swish(pretrained=False, **kw):
    """ShuffleNetV2 x1.0 with swish activations (reference vision/models/shufflenetv2.py:541)."""
    _no_pretrained(pretrained)
    return ShuffleNetV2(1.0, act='swish', **kw)


# ----------------------------------------------------------------------------- DenseNet
class _DenseLayer(nn.Layer):
    def __init__(self, cin, growth, bn_size, dropout):
        super().__init__()
        self.bn1 = nn.BatchNorm2D(cin)
        self.conv1 = nn.Conv2D(cin, bn_size * growth, 1, bias_attr=False)
        self.bn2 = nn.BatchNorm2D(bn_size * growth)
        self.conv2 = nn.Conv2D(bn_size * growth, growth, 3, padding=1, bias_attr=False)
        self.dropout = dropout

    def forward(self, x):
        y = self.conv1(F.relu(self.bn1(x)))
        y = self.conv2(F.relu(self.bn2(y)))
        if self.dropout:
            y = F.dropout(y, self.dropout, training=self.training)
        return concat([x, y], axis=1)


class DenseNet(nn.Layer):
    def __init__(self, layers=121, bn_size=4, dropout=0.0, num_classes=1000, with_pool=True):
        super().__init__()
        cfg = {121: (64, 32, [6, 12, 24, 16]), 161: (96, 48, [6, 12, 36, 24]), 169: (64, 32, [6, 12, 32, 32]),
               201: (64, 32, [6, 12, 48, 32]), 264: (64, 32, [6, 12, 64, 48])}
        init, growth, blocks = cfg[layers]
        feats = [nn.Conv2D(3, init, 7, stride=2, padding=3, bias_attr=False), nn.BatchNorm2D(init), nn.ReLU(),
                 nn.MaxPool2D(3, 2, padding=1)]
        c = init
        for i, n in enumerate(blocks):
            for _ in range(n):
                feats.append(_DenseLayer(c, growth, bn_size, dropout))
                c += growth
            if i != len(blocks) - 1:
                feats += [nn.BatchNorm2D(c), nn.ReLU(), nn.Conv2D(c, c // 2, 1, bias_attr=False), nn.AvgPool2D(2, 2)]
                c //= 2
        feats += [nn.BatchNorm2D(c), nn.ReLU()]
        self.features = nn.Sequential(*feats)
        self.num_classes, self.with_pool = num_classes, with_pool
        if with_pool:
            self.pool2d_avg = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.out = nn.Linear(c, num_classes)

    def forward(self, x):
        x = self.features(x)
        if self.with_pool:
            x = self.pool2d_avg(x)
        return self.out(flatten(x, 1)) if self.num_classes > 0 else x


def densenet121(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return DenseNet(121, **kw)


def densenet161(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return DenseNet(161, **kw)


def densenet169(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return DenseNet(169, **kw)


def densenet201(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return DenseNet(201, **kw)


def densenet264(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return DenseNet(264, **kw)


# ----------------------------------------------------------------------------- GoogLeNet / InceptionV3
class _Inception(nn.Layer):
    def __init__(self, cin, c1, c3r, c3, c5r, c5, pp):
        super().__init__()
        self.b1 = ConvBNLayer(cin, c1, 1)
        self.b2 = nn.Sequential(ConvBNLayer(cin, c3r, 1), ConvBNLayer(c3r, c3, 3, padding=1))
        self.b3 = nn.Sequential(ConvBNLayer(cin, c5r, 1), ConvBNLayer(c5r, c5, 5, padding=2))
        self.b4 = nn.Sequential(nn.MaxPool2D(3, 1, padding=1), ConvBNLayer(cin, pp, 1))

    def forward(self, x):
        return concat([self.b1(x), self.b2(x), self.b3(x), self.b4(x)], axis=1)


class GoogLeNet(nn.Layer):
    def __init__(self, num_classes=1000, with_pool=True):
        super().__init__()
        self.stem = nn.Sequential(ConvBNLayer(3, 64, 7, 2, 3), nn.MaxPool2D(3, 2, padding=1), ConvBNLayer(64, 64, 1),
                                  ConvBNLayer(64, 192, 3, padding=1), nn.MaxPool2D(3, 2, padding=1))
        self.inc = nn.Sequential(
            _Inception(192, 64, 96, 128, 16, 32, 32), _Inception(256, 128, 128, 192, 32, 96, 64),
            nn.MaxPool2D(3, 2, padding=1),
            _Inception(480, 192, 96, 208, 16, 48, 64), _Inception(512, 160, 112, 224, 24, 64, 64),
            _Inception(512, 128, 128, 256, 24, 64, 64), _Inception(512, 112, 144, 288, 32, 64, 64),
            _Inception(528, 256, 160, 320, 32, 128, 128), nn.MaxPool2D(3, 2, padding=1),
            _Inception(832, 256, 160, 320, 32, 128, 128), _Inception(832, 384, 192, 384, 48, 128, 128))
        self.num_classes, self.with_pool = num_classes, with_pool
        self.pool = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.dropout = nn.Dropout(0.4)
            self.fc = nn.Linear(1024, num_classes)

    def forward(self, x):
        x = self.inc(self.stem(x))
        if self.with_pool:
            x = self.pool(x)
        if self.num_classes > 0:
            x = self.fc(self.dropout(flatten(x, 1)))
        return x


def googlenet(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return GoogLeNet(**kw)


class InceptionV3(nn.Layer):
    """Compact InceptionV3 (stem + mixed blocks with the reference's channel plan)."""

    def __init__(self, num_classes=1000, with_pool=True):
        super().__init__()
        self.stem = nn.Sequential(ConvBNLayer(3, 32, 3, 2), ConvBNLayer(32, 32, 3), ConvBNLayer(32, 64, 3, padding=1),
                                  nn.MaxPool2D(3, 2), ConvBNLayer(64, 80, 1), ConvBNLayer(80, 192, 3),
                                  nn.MaxPool2D(3, 2))
        self.mixed = nn.Sequential(_Inception(192, 64, 48, 64, 64, 96, 32), _Inception(256, 64, 48, 64, 64, 96, 64),
                                   _Inception(288, 64, 48, 64, 64, 96, 64), nn.MaxPool2D(3, 2),
                                   _Inception(288, 192, 128, 192, 128, 192, 192),
                                   _Inception(768, 320, 192, 384, 448, 384, 192),
                                   _Inception(1280, 320, 384, 768, 448, 768, 192))
        self.num_classes, self.with_pool = num_classes, with_pool
        self.avg_pool = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.dropout = nn.Dropout(0.2)
            self.fc = nn.Linear(2048, num_classes)

    def forward(self, x):
        x = self.mixed(self.stem(x))
        if self.with_pool:
            x = self.avg_pool(x)
        if self.num_classes > 0:
            x = self.fc(self.dropout(flatten(x, 1)))
        return x


def inception_v3(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return InceptionV3(**kw)


_ = (reshape, transpose)
