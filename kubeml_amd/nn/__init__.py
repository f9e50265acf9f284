"""MI355X-native layers: NHWC bf16 activations on HIP kernels, flat fp32 params."""
from .flat import FlatParamSpace, flatten_module, grad_storage_of, master_of, shadow_of
from .modules import (AdaptiveAvgPool2d, BatchNorm2d, Conv2d, CrossEntropyLoss, Flatten, Linear, MaxPool2d, ReLU,
                      backward_loss, cross_entropy, to_nhwc)

__all__ = ["FlatParamSpace", "flatten_module", "grad_storage_of", "master_of", "shadow_of", "AdaptiveAvgPool2d",
           "BatchNorm2d", "Conv2d", "CrossEntropyLoss", "Flatten", "Linear", "MaxPool2d", "ReLU", "backward_loss",
           "cross_entropy",
           "to_nhwc"]
