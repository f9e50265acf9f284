"""LeNet-5 as shipped in the reference's MNIST function
(ml/experiments/kubeml/function_lenet.py:14-50) — including the ReLU after the last
Linear (a quirk preserved for parity).  44,426 parameters,
10 state_dict tensors, same names as the reference's module.

On a GPU it runs on the MI355X layers: NHWC bf16 activations with channels padded
to 8 (conv1's 6 output channels carry 2 zero channels into conv2, whose padded
input channels they fill), MFMA implicit-GEMM convs, the max-pool kernel, and the
MFMA linear layers with ReLU fused into their epilogue.  On CPU the same modules run
stock fp32 torch ops.
"""
from __future__ import annotations

import torch.nn as tnn

from ..nn.modules import Conv2d, Flatten, Linear, MaxPool2d, ReLU, to_nhwc


class LeNet(tnn.Module):
    def __init__(self, num_classes: int = 10):
        super().__init__()
        self.conv1 = Conv2d(1, 6, 5)
        self.relu1 = ReLU()
        self.pool1 = MaxPool2d(2)
        self.conv2 = Conv2d(6, 16, 5)
        self.relu2 = ReLU()
        self.pool2 = MaxPool2d(2)
        self.fc1 = Linear(256, 120, fused_relu=True)
        self.relu3 = ReLU()
        self.fc2 = Linear(120, 84, fused_relu=True)
        self.relu4 = ReLU()
        self.fc3 = Linear(84, num_classes, fused_relu=True)
        self.relu5 = ReLU()
        self.flatten = Flatten()

    def forward(self, x):
        """x: [B, 1, 28, 28] (NCHW, as the reference's transforms produce) or NHWC."""
        if x.dim() == 4 and x.shape[1] == 1 and x.shape[-1] != 1:
            x = to_nhwc(x, 8 if x.is_cuda else None)
        y = self.pool1(self.relu1(self.conv1(x)))
        y = self.pool2(self.relu2(self.conv2(y)))
        y = self.flatten(y)
        # fc1..fc3 apply their ReLU in the GEMM epilogue (relu3..relu5 of the reference)
        return self.fc3(self.fc2(self.fc1(y)))
