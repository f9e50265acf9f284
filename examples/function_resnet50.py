"""ResNet-50 / ImageNet-shaped data with K-step local SGD (north-star config 3).

The reference ships no ResNet-50 function; this is its ResNet-34 function
(ml/experiments/kubeml/function_resnet34.py:47-104) on the Bottleneck model and
ImageNet-sized images: torchvision-layout resnet50 (1000 classes), SGD momentum 0.9 /
wd 1e-4, horizontal flip + ImageNet normalisation on device (synthetic uint8 224x224
images: no network for ImageNet).  Run it with ``kubeml train --K 8`` (or any K > 1):
every K minibatches the workers' models are averaged — the reference's K-AVG round
(python/kubeml/kubeml/network.py:289-306) as one all-reduce of the flat state buffer.

``ASYNC_KAVG = True`` opts into the overlapped (staleness-1) average of SURVEY §5.8.5: the
all-reduce of round r runs on a comm stream while round r+1 computes, and its result is
applied one round late (parallel/kavg.py AsyncModelAverager); the job history records it.
"""
from typing import Tuple

import torch
from torch.optim import SGD

from kubeml import KubeModel
from kubeml_amd.models.resnet import resnet50
from kubeml_amd.sdk.vision import IMAGENET_MEAN, IMAGENET_STD, ImageDataset, prepare


class ImageNetShaped(ImageDataset):
    def __init__(self, name="imagenet_synth"):
        super().__init__(name, mean=IMAGENET_MEAN, std=IMAGENET_STD, crop_pad=0, flip=True)


class KubeResnet50(KubeModel):
    ASYNC_KAVG = False

    def __init__(self, network, dataset):
        super().__init__(network, dataset, gpu=True)

    def configure_optimizers(self) -> torch.optim.Optimizer:
        return SGD(self.parameters(), lr=self.lr, momentum=0.9, weight_decay=1e-4)

    def train(self, batch, batch_index) -> float:
        x, y = prepare(batch, self._dataset, train=True, seed=self.args._func_id)
        return self.step(x, y)  # one hipGraph replay; device loss (no host sync)

    def validate(self, batch, batch_index) -> Tuple[float, float]:
        x, y = prepare(batch, self._dataset, train=False)
        correct, loss = self.evaluate(x, y)  # graph-replayed eval forward on the GPU
        return correct * 100 / self.batch_size, loss

    def infer(self, data):
        x = torch.tensor(data, dtype=torch.uint8, device=self.device)
        x, _ = prepare((x, torch.zeros(len(x), dtype=torch.int64, device=self.device)), self._dataset, train=False)
        return self(x).float().argmax(1)


def main():
    return KubeResnet50(resnet50(1000), ImageNetShaped()).start()
