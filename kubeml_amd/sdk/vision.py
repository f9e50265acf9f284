"""Image-classification helpers for user functions (CIFAR/MNIST-style datasets).

The reference's CIFAR functions run torchvision transforms per sample in a
``DataLoader`` (function_resnet34.py:17-44).  On MI355X that host path would cap a
worker far below the GPU's rate, so :class:`ImageDataset` hands whole uint8 batches
to the device (``collate_batch``) and :func:`prepare` runs the fused augmentation
kernel there (random crop with zero padding, horizontal flip, normalisation, NHWC
bf16 with channels padded to 8).  On CPU workers the same code falls back to the
numpy/torch transforms with identical semantics, so functions stay portable.
"""
from __future__ import annotations

from typing import Sequence, Tuple

import numpy as np
import torch

from .dataset import KubeDataset

CIFAR10_MEAN, CIFAR10_STD = (0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010)
IMAGENET_MEAN, IMAGENET_STD = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)


class ImageDataset(KubeDataset):
    """uint8 ``[N, H, W, C]`` images + integer labels; batches are ``(uint8 tensor, int64 labels)``."""

    def __init__(self, dataset: str, mean: Sequence[float] = IMAGENET_MEAN, std: Sequence[float] = IMAGENET_STD,
                 crop_pad: int = 4, flip: bool = True):
        super().__init__(dataset)
        self.mean, self.std = tuple(mean), tuple(std)
        self.crop_pad, self.flip = crop_pad, flip

    def collate_batch(self, data: np.ndarray, labels: np.ndarray):
        x = torch.from_numpy(np.ascontiguousarray(data))
        if x.dim() == 3:  # [N, H, W] grayscale
            x = x.unsqueeze(-1)
        y = torch.from_numpy(np.ascontiguousarray(labels).reshape(-1).astype(np.int64))
        return x, y

    def __getitem__(self, i):
        return self.data[i], int(self.labels[i])

    def __len__(self):
        return len(self.data) if self.data is not None else 0


_CTRS = {}


def prepare(batch: Tuple[torch.Tensor, torch.Tensor], ds: ImageDataset, train: bool, seed: int = 0):
    """Device batch → (model input, labels).  GPU: one fused augment kernel launch;
    CPU: the same ops in torch (NCHW float32)."""
    x, y = batch
    if x.is_cuda:
        from ..ops import kernels as K
        key = (x.device, seed)
        ctr = _CTRS.get(key)
        if ctr is None:
            ctr = torch.tensor([float(seed), 0.0, 0.0], dtype=torch.float32, device=x.device)
            _CTRS[key] = ctr
        if x.dtype != torch.uint8:
            raise TypeError("GPU augmentation expects uint8 images")
        B = x.shape[0]
        xb, yb = K.augment(x.contiguous(), y.contiguous(), ctr, B, pad=ds.crop_pad if train else 0,
                           flip=ds.flip and train, train=train, mean=ds.mean, std=ds.std)
        K.advance_counter_(ctr, B, B)
        return xb, yb
    xf = x.permute(0, 3, 1, 2).float().div_(255.0)
    if train:
        p = ds.crop_pad
        if p:
            B, C, H, W = xf.shape
            xp = torch.nn.functional.pad(xf, (p, p, p, p))
            ii = torch.randint(0, 2 * p + 1, (B,))
            jj = torch.randint(0, 2 * p + 1, (B,))
            xf = torch.stack([xp[b, :, ii[b]:ii[b] + H, jj[b]:jj[b] + W] for b in range(B)])
        if ds.flip:
            m = torch.rand(xf.shape[0]) < 0.5
            xf[m] = xf[m].flip(-1)
    mean = torch.tensor(ds.mean[: xf.shape[1]]).view(1, -1, 1, 1)
    std = torch.tensor(ds.std[: xf.shape[1]]).view(1, -1, 1, 1)
    return (xf - mean) / std, y
