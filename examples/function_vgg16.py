"""VGG-16-BN / CIFAR-100 (north-star config 4).  The reference's VGG function
(ml/experiments/kubeml/function_vgg11.py) used torchvision vgg11 with Adam on an older
KubeModel API; this is the same family on the current API: Adam(lr), CIFAR-100
mean/std from the recipe it cites, crop+flip augmentation on device."""
from typing import Tuple

import torch
from torch.optim import Adam

from kubeml import KubeModel
from kubeml_amd.models.vgg import vgg16
from kubeml_amd.sdk.vision import ImageDataset, prepare

CIFAR100_MEAN = (0.5070751592371323, 0.48654887331495095, 0.4409178433670343)
CIFAR100_STD = (0.2673342858792401, 0.2564384629170883, 0.27615047132568404)


class Cifar100Dataset(ImageDataset):
    def __init__(self):
        super().__init__("cifar100", mean=CIFAR100_MEAN, std=CIFAR100_STD)


class KubeVGG(KubeModel):
    def __init__(self, network, dataset):
        super().__init__(network, dataset, gpu=True)

    def configure_optimizers(self) -> torch.optim.Optimizer:
        return Adam(self.parameters(), lr=self.lr)

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
    return KubeVGG(vgg16(100), Cifar100Dataset()).start()
