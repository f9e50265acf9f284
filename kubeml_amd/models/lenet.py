"""LeNet-5 as shipped in the reference's MNIST function
(ml/experiments/kubeml/function_lenet.py:14-50) — including the ReLU after the last
Linear (a quirk preserved for parity).  44,426 parameters,
10 state_dict tensors.  Plain torch.nn: it is user-model code and north-star config 1
runs it on CPU workers."""
from __future__ import annotations

import torch.nn as nn


class LeNet(nn.Module):
    def __init__(self, num_classes: int = 10):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 6, 5)
        self.relu1 = nn.ReLU()
        self.pool1 = nn.MaxPool2d(2)
        self.conv2 = nn.Conv2d(6, 16, 5)
        self.relu2 = nn.ReLU()
        self.pool2 = nn.MaxPool2d(2)
        self.fc1 = nn.Linear(256, 120)
        self.relu3 = nn.ReLU()
        self.fc2 = nn.Linear(120, 84)
        self.relu4 = nn.ReLU()
        self.fc3 = nn.Linear(84, num_classes)
        self.relu5 = nn.ReLU()

    def forward(self, x):
        y = self.pool1(self.relu1(self.conv1(x)))
        y = self.pool2(self.relu2(self.conv2(y)))
        y = y.view(y.shape[0], -1)
        y = self.relu3(self.fc1(y))
        y = self.relu4(self.fc2(y))
        return self.relu5(self.fc3(y))
