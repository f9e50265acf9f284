"""ResNet-34 / CIFAR-10 function — the reference's headline workload
(ml/experiments/kubeml/function_resnet34.py): torchvision-layout resnet34 with the
ImageNet stem and 1000-class head, SGD(lr, wd 1e-4), LR x0.1 after epoch 80 (the
reference's never-firing x0.01 branch kept as written),
RandomCrop(32, 4) + RandomHorizontalFlip + Normalize(ImageNet mean/std), accuracy
= correct * 100 / batch_size.

MI355X-native data path: whole uint8 batches go to HBM and one fused kernel does
crop/flip/normalise into NHWC bf16; forward+loss+backward+SGD of a batch is one
hipGraph replay (``self.step``).  Runs unchanged on CPU workers (stock ops).
"""
from typing import Tuple

import torch
from torch.optim import SGD

from kubeml import KubeModel
from kubeml_amd.models.resnet import resnet34
from kubeml_amd.sdk.vision import IMAGENET_MEAN, IMAGENET_STD, ImageDataset, prepare


class Cifar10Dataset(ImageDataset):
    def __init__(self):
        super().__init__("cifar10", mean=IMAGENET_MEAN, std=IMAGENET_STD, crop_pad=4, flip=True)


class KubeResnet34(KubeModel):
    def __init__(self, network, dataset):
        super().__init__(network, dataset, gpu=True)

    def configure_optimizers(self) -> torch.optim.Optimizer:
        # the reference's schedule, quirk included (function_resnet34.py:57-60): the `elif`
        # can never fire (epoch > 120 implies epoch > 80), so the LR stays at x0.1 after 80
        lr = self.lr
        if self.epoch > 80:
            lr *= 0.1
        elif self.epoch > 120:
            lr *= 0.01
        return SGD(self.parameters(), lr=lr, weight_decay=1e-4)

    def train(self, batch, batch_index) -> float:
        x, y = prepare(batch, self._dataset, train=True, seed=self.args._func_id)
        return self.step(x, y)  # device tensor: no host sync per batch

    def validate(self, batch, batch_index) -> Tuple[float, float]:
        x, y = prepare(batch, self._dataset, train=False)
        correct, loss = self.evaluate(x, y)  # graph-replayed eval forward on the GPU
        return correct * 100 / self.batch_size, loss

    def infer(self, data):
        x = torch.tensor(data, dtype=torch.uint8, device=self.device)
        x, _ = prepare((x, torch.zeros(x.shape[0], dtype=torch.int64, device=self.device)), self._dataset,
                       train=False)
        return self(x).float().argmax(1)


def main():
    resnet = resnet34()
    dataset = Cifar10Dataset()
    kubenet = KubeResnet34(resnet, dataset)
    return kubenet.start()
