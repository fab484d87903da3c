"""Model zoo: the reference's workloads (CIFAR 7-layer CNN, BiCNN QA) and the
BASELINE.json configs (LeNet, ResNet-50, AlexNet, VGG-16)."""
from .resnet import ResNet, resnet18, resnet34, resnet50, resnet101, resnet152

_REGISTRY = {
    "resnet18": resnet18,
    "resnet34": resnet34,
    "resnet50": resnet50,
    "resnet101": resnet101,
    "resnet152": resnet152,
}


def register(name):
    def deco(fn):
        _REGISTRY[name] = fn
        return fn

    return deco


def get_model(name: str, **kw):
    try:
        fn = _REGISTRY[name]
    except KeyError:
        raise ValueError(f"unknown model {name!r}; have {sorted(_REGISTRY)}") from None
    return fn(**kw)


from . import cnn  # noqa: E402,F401  (registers lenet / cnn7 / alexnet / vgg16)
