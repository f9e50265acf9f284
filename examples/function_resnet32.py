"""CIFAR ResNet-32 (option-A shortcuts) — reference ml/experiments/kubeml/resnet32.py:
SGD(momentum .9, wd 1e-4), LR /10 from epoch 100, CIFAR-10 mean/std, crop+flip.
Used for the K-sweep figures of the reference paper."""
from typing import Tuple

import torch
from torch.optim import SGD

from kubeml import KubeModel
from kubeml_amd.models.resnet import resnet32
from kubeml_amd.sdk.vision import CIFAR10_MEAN, CIFAR10_STD, ImageDataset, prepare


class Cifar10Dataset(ImageDataset):
    def __init__(self):
        super().__init__("cifar10", mean=CIFAR10_MEAN, std=CIFAR10_STD)


class KubeResnet(KubeModel):
    def __init__(self, network, dataset):
        super().__init__(network, dataset, gpu=True)

    def configure_optimizers(self) -> torch.optim.Optimizer:
        lr = self.lr / 10 if self.epoch >= 100 else self.lr
        return SGD(self.parameters(), lr=lr, momentum=0.9, weight_decay=1e-4)

    def train(self, batch, batch_index) -> float:
        x, y = prepare(batch, self._dataset, train=True, seed=self.args._func_id)
        return self.step(x, y)  # device tensor: no host sync per batch

    def validate(self, batch, batch_index) -> Tuple[float, float]:
        x, y = prepare(batch, self._dataset, train=False)
        correct, loss = self.evaluate(x, y)  # graph-replayed eval forward on the GPU
        return correct * 100 / self.batch_size, loss

    def infer(self, data):
        x = torch.tensor(data, dtype=torch.uint8, device=self.device)
        x, _ = prepare((x, torch.zeros(len(x), dtype=torch.int64, device=self.device)), self._dataset, train=False)
        return self(x).float().argmax(1)


def main():
    torch.manual_seed(42)
    return KubeResnet(resnet32(), Cifar10Dataset()).start()
