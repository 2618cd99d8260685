"""Model zoo for the benchmarks (architectures only; random init, synthetic data)."""
from .bert import bert_base  # noqa: F401
from .lstm import lstm_ptb  # noqa: F401
from .resnet import resnet18, resnet18_cifar, resnet34, resnet50, resnet101  # noqa: F401
from .resnet9 import resnet9  # noqa: F401
from .vgg import vgg16  # noqa: F401

MODELS = {
    "resnet18": resnet18, "resnet18_cifar": resnet18_cifar, "resnet34": resnet34, "resnet50": resnet50,
    "resnet101": resnet101, "resnet9": resnet9, "vgg16": vgg16, "lstm_ptb": lstm_ptb, "bert_base": bert_base,
}
