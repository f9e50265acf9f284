"""The torchvision transforms the reference's functions use, without torchvision
(not available on the target image): ``Compose``, ``ToTensor``, ``Normalize``,
``RandomHorizontalFlip``, ``RandomCrop(size, padding)``, ``ToPILImage`` (identity on
arrays).  Semantics follow torchvision on HWC uint8 numpy input
(function_lenet.py:57-60, function_resnet34.py:17-30).

These are the per-sample CPU path (CPU workers, parity tests).  The GPU path for the
CIFAR functions is the fused on-device ``kml_augment`` kernel
(:func:`kubeml_amd.ops.kernels.augment`) fed by ``KubeDataset.collate_batch``.
"""
from __future__ import annotations

import random
from typing import Sequence

import numpy as np
import torch


class Compose:
    def __init__(self, ts):
        self.ts = list(ts)

    def __call__(self, x):
        for t in self.ts:
            x = t(x)
        return x


class ToPILImage:
    """Identity on HWC arrays (the pipeline stays in numpy)."""

    def __call__(self, x):
        return np.asarray(x)


class ToTensor:
    """HWC (or HW) uint8 → CHW float in [0, 1]; float arrays are not rescaled."""

    def __call__(self, x):
        if isinstance(x, torch.Tensor):
            return x
        a = np.asarray(x)
        if a.ndim == 2:
            a = a[:, :, None]
        t = torch.from_numpy(np.ascontiguousarray(a.transpose(2, 0, 1)))
        if a.dtype == np.uint8:
            return t.float().div_(255.0)
        return t.float()


class Normalize:
    def __init__(self, mean: Sequence[float], std: Sequence[float]):
        self.mean = torch.tensor(mean, dtype=torch.float32).view(-1, 1, 1)
        self.std = torch.tensor(std, dtype=torch.float32).view(-1, 1, 1)

    def __call__(self, t: torch.Tensor):
        return (t - self.mean) / self.std


class RandomHorizontalFlip:
    def __init__(self, p: float = 0.5):
        self.p = p

    def __call__(self, x):
        if random.random() < self.p:
            if isinstance(x, torch.Tensor):
                return x.flip(-1)
            return np.ascontiguousarray(np.asarray(x)[:, ::-1])
        return x


class RandomCrop:
    def __init__(self, size, padding: int = 0):
        self.size = (size, size) if isinstance(size, int) else tuple(size)
        self.padding = padding

    def __call__(self, x):
        a = np.asarray(x)
        p = self.padding
        if p:
            pad = ((p, p), (p, p)) + (((0, 0),) if a.ndim == 3 else ())
            a = np.pad(a, pad)
        h, w = a.shape[:2]
        th, tw = self.size
        i = random.randint(0, h - th)
        j = random.randint(0, w - tw)
        return a[i:i + th, j:j + tw]
