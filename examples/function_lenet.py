"""LeNet-5 / MNIST function — the reference's ml/experiments/kubeml/function_lenet.py
ported to this framework: same network (incl. ReLU after fc3), same SGD(momentum .9,
wd 1e-4), same per-batch accuracy definition.  torchvision is replaced by
kubeml_amd.data.transforms (identical ToTensor/Normalize semantics).

    kubeml fn create --name lenet --code examples/function_lenet.py
    kubeml train -f lenet -d mnist -e 5 -b 64 --lr 0.01 --parallelism 2 --K 8
"""
import logging
from typing import Tuple

import torch
import torch.nn as nn
from torch.optim import SGD

from kubeml import KubeDataset, KubeModel
from kubeml_amd.data import transforms
from kubeml_amd.models.lenet import LeNet


class MnistDataset(KubeDataset):
    def __init__(self):
        super().__init__("mnist")
        self.transf = transforms.Compose([transforms.ToTensor(), transforms.Normalize((0.1307,), (0.3081,))])

    def __getitem__(self, index):
        x = self.data[index]
        y = self.labels[index]
        return self.transf(x), y.astype("int64")

    def __len__(self):
        return len(self.data)


class KubeLeNet(KubeModel):
    def __init__(self, network: nn.Module, dataset: MnistDataset):
        super().__init__(network, dataset, gpu=True)

    def configure_optimizers(self) -> torch.optim.Optimizer:
        return SGD(self.parameters(), lr=self.lr, momentum=0.9, weight_decay=1e-4)

    def init(self):
        pass

    def train(self, batch, batch_index) -> float:
        criterion = nn.CrossEntropyLoss()
        x, y = batch
        self.optimizer.zero_grad()
        output = self(x)
        loss = criterion(output, y)
        loss.backward()
        self.optimizer.step()
        if batch_index % 10 == 0:
            logging.info(f"Index {batch_index}, error: {loss.item()}")
        return loss.item()

    def validate(self, batch, batch_index) -> Tuple[float, float]:
        criterion = nn.CrossEntropyLoss()
        x, y = batch
        output = self(x)
        _, predicted = torch.max(output.data, 1)
        test_loss = criterion(output, y).item()
        correct = predicted.eq(y).sum().item()
        accuracy = correct * 100 / self.batch_size   # reference quirk: divides by batch_size
        return accuracy, test_loss

    def infer(self, data):
        x = torch.tensor(data, dtype=torch.float32, device=self.device)
        if x.dim() == 3:
            x = x.unsqueeze(1)
        return self(x).argmax(1)


def main():
    torch.manual_seed(42)
    lenet = LeNet()
    dataset = MnistDataset()
    kubenet = KubeLeNet(lenet, dataset)
    return kubenet.start()
