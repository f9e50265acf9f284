"""VGG-11/16 (+BN) on the MI355X layers — north-star config 4 (VGG-16 / CIFAR-100) and
the reference's VGG-11 function (ml/experiments/kubeml/function_vgg11.py:10-12 uses
``torchvision.models.vgg11``).

``state_dict`` names follow torchvision (``features.<i>.*``, ``classifier.<i>.*``) so
checkpoints interoperate.  Two heads:

* ``head="imagenet"`` — torchvision's: AdaptiveAvgPool2d(7) + 25088→4096→4096→classes.
  On 32×32 CIFAR input the feature map is 1×1 and the 7×7 pool is a replication;
* ``head="cifar"`` (default for the CIFAR configs) — 512→4096→4096→classes, as in the
  pytorch-cifar100 recipe the reference cites (function_vgg11.py:14-15).

Activations are NHWC bf16 on the GPU.  In GPU training the Conv→BN→ReLU units between two
max-pools run as one fused autograd node (nn/fused.py ``BlockFn``, the ResNet blocks'
executor): conv (MFMA implicit GEMM, +bias) with the BN statistics in its epilogue, one
BN-apply+ReLU pass; backward: BN backward, then dgrad + wgrad as one grouped launch whose dgrad
epilogue already emits the next BatchNorm's dgamma/dbeta partial rows.  The classifier's
Linear+ReLU pairs run with the ReLU in the GEMM epilogue.  The classifier's
dropout is the in-tree counter-hash kernel (nn/transformer.py ``Dropout``: the mask is a hash of
(seed, step, layer salt, index), recomputed in the backward, nothing stored); its step counter
advances once per training forward on the device, so a replayed hipGraph draws a new mask.
"""
from __future__ import annotations

from typing import List, Union

import torch
import torch.nn as tnn

from ..nn.fused import BlockFn, block_params, refresh_transposed
from ..nn.modules import BatchNorm2d, Conv2d, Flatten, Linear, MaxPool2d, ReLU, to_nhwc
from ..nn.transformer import Dropout, RNGState


class _Stage:
    """Conv→BN→ReLU units between two max-pools (plain holder: the modules stay registered under
    ``features`` with torchvision's names); ``BlockFn`` runs the plan."""

    def __init__(self, units):
        self._kml_plan = [(conv, bn, True, "main") for conv, bn in units]


def _segments(features: tnn.Sequential):
    """[(stage | None, pool | None)]: the fused stages and the max-pools of a BN feature stack, or
    None when the stack is not made of Conv→BN→ReLU units and pools."""
    mods = list(features)
    segs, units, i = [], [], 0
    while i < len(mods):
        m = mods[i]
        if isinstance(m, Conv2d) and i + 2 < len(mods) and isinstance(mods[i + 1], BatchNorm2d) and \
                isinstance(mods[i + 2], ReLU):
            units.append((m, mods[i + 1]))
            i += 3
        elif isinstance(m, MaxPool2d):
            segs.append((_Stage(units) if units else None, m))
            units = []
            i += 1
        else:
            return None
    if units:
        segs.append((_Stage(units), None))
    return segs

CFGS = {
    "vgg11": [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "vgg13": [64, 64, "M", 128, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "vgg16": [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
}


def make_features(cfg: List[Union[int, str]], batch_norm: bool, in_ch: int = 3) -> tnn.Sequential:
    layers = []
    c = in_ch
    for v in cfg:
        if v == "M":
            layers.append(MaxPool2d(2, 2))
        else:
            layers.append(Conv2d(c, v, 3, padding=1))
            if batch_norm:
                layers.append(BatchNorm2d(v))
            layers.append(ReLU(inplace=True))
            c = v
    return tnn.Sequential(*layers)


class _Replicate7(tnn.Module):
    """AdaptiveAvgPool2d((7, 7)) on a 1x1 map = replicate (torchvision head on CIFAR)."""

    def forward(self, x):
        B, H, W, C = x.shape
        if (H, W) == (7, 7):
            return x
        if (H, W) != (1, 1):
            raise NotImplementedError("imagenet head expects 1x1 or 7x7 feature maps")
        return x.expand(B, 7, 7, C).contiguous()


class VGG(tnn.Module):
    def __init__(self, cfg: str = "vgg16", batch_norm: bool = True, num_classes: int = 100, head: str = "cifar",
                 dropout: float = 0.5):
        super().__init__()
        self.features = make_features(CFGS[cfg], batch_norm)
        self.head = head
        if head == "imagenet":
            self.avgpool = _Replicate7()
            fin = 512 * 7 * 7
        else:
            self.avgpool = None
            fin = 512
        self.flatten = Flatten()
        self.rng = RNGState(seed=17)
        self.classifier = tnn.Sequential(
            Linear(fin, 4096, fused_relu=True), ReLU(True), Dropout(dropout, rng=self.rng),
            Linear(4096, 4096, fused_relu=True), ReLU(True), Dropout(dropout, rng=self.rng),
            Linear(4096, num_classes))
        object.__setattr__(self, "_kml_segments", _segments(self.features) if batch_norm else None)
        for m in self.modules():
            if isinstance(m, Conv2d):
                tnn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
                if m.bias is not None:
                    tnn.init.zeros_(m.bias)
            elif isinstance(m, BatchNorm2d):
                tnn.init.ones_(m.weight)
                tnn.init.zeros_(m.bias)
            elif isinstance(m, Linear):
                tnn.init.normal_(m.weight, 0, 0.01)
                tnn.init.zeros_(m.bias)

    def _features(self, x):
        mods = list(self.features)
        i = 0
        while i < len(mods):
            m = mods[i]
            if isinstance(m, BatchNorm2d) and i + 1 < len(mods) and isinstance(mods[i + 1], ReLU):
                x = m(x, relu=True)  # fused BN-apply + ReLU
                i += 2
                continue
            x = m(x)
            i += 1
        return x

    def _features_fused(self, x):
        from ..ops import kernels as K
        sp = getattr(self, "_kml_flat", None)
        if sp is not None and sp.i64_buffers:
            K.add_i64_(sp.i64_arena_now())     # every BN's num_batches_tracked, one launch
        else:
            for m in self.features:
                if isinstance(m, BatchNorm2d):
                    K.add_i64_(m.num_batches_tracked)
        convs = getattr(self, "_kml_convs", None)
        if convs is None:
            convs = [m for m in self.features if isinstance(m, Conv2d)]
            object.__setattr__(self, "_kml_convs", convs)
        refresh_transposed(convs)
        for stage, pool in self._kml_segments:
            if stage is not None:
                x = BlockFn.apply(x, stage, *block_params(stage))
            if pool is not None:
                x = pool(x)
        return x

    def _stage_features(self, x):
        fused = x.is_cuda and self.training and torch.is_grad_enabled() and self._kml_segments is not None
        if self.training and x.is_cuda:
            self.rng.advance(x.device)      # a fresh dropout mask per step (device counter)
        x = to_nhwc(x, 8)
        return self._features_fused(x) if fused else self._features(x)

    def _stage_head(self, x):
        if self.avgpool is not None:
            x = self.avgpool(x)
        x = self.flatten(x)
        if not x.is_cuda:
            return self.classifier(x)
        mods = list(self.classifier)
        for i, m in enumerate(mods):
            if isinstance(m, ReLU) and i > 0 and getattr(mods[i - 1], "fused_relu", False):
                continue                      # already applied in the Linear's epilogue
            x = m(x)
        return x

    def forward(self, x):
        return self._stage_head(self._stage_features(x))

    def stages(self):
        """[features, head] for a stage-split step (engine/staged.py): backward finishes the
        classifier's gradients first — 19.3 M of VGG-16's 34.0 M parameters with the CIFAR head —
        so a per-stage optimizer (``make_train_step(opt_overlap=True)``) updates them on a side
        stream while the convolutions run backward."""
        return [self._stage_features, self._stage_head]

    def stage_params(self):
        """Parameters owned by each stage of :meth:`stages` (one contiguous flat range each)."""
        return [list(self.features.parameters()), list(self.classifier.parameters())]


def vgg11(num_classes: int = 1000, batch_norm: bool = False, head: str = "imagenet", **kw) -> VGG:
    """torchvision ``vgg11()`` layout (the reference's VGG-11 function)."""
    return VGG("vgg11", batch_norm, num_classes, head, **kw)


def vgg11_bn(num_classes: int = 100, head: str = "cifar", **kw) -> VGG:
    return VGG("vgg11", True, num_classes, head, **kw)


def vgg16(num_classes: int = 100, batch_norm: bool = True, head: str = "cifar", **kw) -> VGG:
    """VGG-16-BN / CIFAR-100 (north-star config 4)."""
    return VGG("vgg16", batch_norm, num_classes, head, **kw)


vgg16_bn = vgg16
