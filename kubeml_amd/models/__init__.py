"""Model zoo (MI355X-native layers; torchvision-compatible state_dict names).

Workloads shipped by the reference and the north-star configs:
  lenet       LeNet-5 / MNIST           (ml/experiments/kubeml/function_lenet.py)
  resnet34    ResNet-34 / CIFAR-10      (function_resnet34.py) — headline benchmark
  resnet32    CIFAR ResNet-32           (resnet32.py)
  resnet50    ResNet-50 / ImageNet-shape (north-star config 3)
  vgg16       VGG-16-BN / CIFAR-100     (north-star config 4; function_vgg11.py family)
  bert_base   BERT-base MLM             (north-star config 5)
"""
from __future__ import annotations


def get_model(name: str, **kw):
    name = name.lower()
    if name in ("resnet18", "resnet34", "resnet50"):
        from . import resnet
        return getattr(resnet, name)(**kw)
    if name in ("resnet20", "resnet32", "resnet44", "resnet56"):
        from . import resnet
        return getattr(resnet, name)(**kw)
    if name == "lenet":
        from .lenet import LeNet
        return LeNet(**kw)
    if name in ("vgg11", "vgg16"):
        from . import vgg
        return getattr(vgg, name)(**kw)
    if name in ("bert_base", "bert"):
        from .bert import bert_base_mlm
        return bert_base_mlm(**kw)
    raise KeyError(f"unknown model {name!r}")
