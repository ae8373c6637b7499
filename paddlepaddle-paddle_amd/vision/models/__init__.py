"""paddle.vision.models (reference: python/paddle/vision/models/__init__.py)."""
from .lenet import LeNet  # noqa: F401
from .resnet import (ResNet, BasicBlock, BottleneckBlock, resnet18, resnet34, resnet50, resnet101, resnet152,  # noqa: F401
                     resnext50_32x4d, resnext50_64x4d, resnext101_32x4d, resnext101_64x4d, resnext152_32x4d,
                     resnext152_64x4d, wide_resnet50_2, wide_resnet101_2)
from .zoo import (VGG, vgg11, vgg13, vgg16, vgg19, AlexNet, alexnet, MobileNetV1, MobileNetV2, MobileNetV3Small,  # noqa: F401
                  MobileNetV3Large, mobilenet_v1, mobilenet_v2, mobilenet_v3_small, mobilenet_v3_large, SqueezeNet,
                  squeezenet1_0, squeezenet1_1, ShuffleNetV2, shufflenet_v2_x0_5, shufflenet_v2_x1_0,
                  shufflenet_v2_x2_0, shufflenet_v2_x0_25, shufflenet_v2_x0_33, shufflenet_v2_x1_5, shufflenet_v2_swish, DenseNet, densenet121, densenet161, densenet169, densenet201, densenet264,
                  GoogLeNet, googlenet, InceptionV3, inception_v3)
