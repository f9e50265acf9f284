"""Layer-by-layer drift of the HIP ResNet-34 vs an fp64 reference (and bf16 autocast).

Separates numerical drift (bf16 activations) from bugs: a bug shows as a jump at one
stage, precision as smooth growth comparable to stock bf16 autocast.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from kubeml_amd.models import torch_reference as R
from kubeml_amd.models.resnet import resnet34
from kubeml_amd.nn import flatten_module


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm()).item()


def stages_ref(m, x):
    out = {}
    x = m.maxpool(m.relu(m.bn1(m.conv1(x))))
    out["stem"] = x
    for n in ["layer1", "layer2", "layer3", "layer4"]:
        x = getattr(m, n)(x)
        out[n] = x
    out["logits"] = m.fc(torch.flatten(m.avgpool(x), 1))
    return out


def stages_ours(m, x):
    out = {}
    x = m._stem_gpu(x)
    out["stem"] = x.permute(0, 3, 1, 2)
    for n in ["layer1", "layer2", "layer3", "layer4"]:
        x = getattr(m, n)(x)
        out[n] = x.permute(0, 3, 1, 2)
    out["logits"] = m.fc(m.avgpool(x))
    return out


def main():
    dev = "cuda"
    torch.manual_seed(0)
    ref = R.resnet34(1000).to(dev)
    ours = resnet34(1000).to(dev)
    ours.load_state_dict(ref.state_dict())
    flatten_module(ours)
    x = torch.randn(32, 3, 32, 32, device=dev).to(torch.bfloat16).float()
    ref64 = R.resnet34(1000).to(dev).double()
    ref64.load_state_dict(ref.state_dict())
    for mode in ["train", "eval"]:
        getattr(ref64, mode)()
        getattr(ref, mode)()
        getattr(ours, mode)()
        with torch.no_grad():
            r64 = stages_ref(ref64, x.double())
            with torch.autocast("cuda", dtype=torch.bfloat16):
                rbf = stages_ref(ref, x)
            from kubeml_amd.nn import to_nhwc
            if mode == "train":
                ours._arena.begin(x.device)
            o = stages_ours(ours, to_nhwc(x, 8))
        for k in r64:
            print(f"{mode:5s} {k:7s} ours {rel(o[k], r64[k]):.4f}   autocast-bf16 {rel(rbf[k], r64[k]):.4f}")


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def grads():
    """Per-parameter gradient error vs fp64, ours vs stock bf16 autocast."""
    dev = "cuda"
    from kubeml_amd.nn import cross_entropy
    torch.manual_seed(0)
    ref = R.resnet34(1000).to(dev)
    ours = resnet34(1000).to(dev)
    ours.load_state_dict(ref.state_dict())
    flatten_module(ours)
    ref64 = R.resnet34(1000).to(dev).double()
    ref64.load_state_dict(ref.state_dict())
    x = torch.randn(32, 3, 32, 32, device=dev).to(torch.bfloat16).float()
    y = torch.randint(0, 1000, (32,), device=dev)
    F.cross_entropy(ref64(x.double()), y).backward()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        lr = ref(x)
    F.cross_entropy(lr.float(), y).backward()
    cross_entropy(ours(x), y).backward()
    p64 = dict(ref64.named_parameters())
    pbf = dict(ref.named_parameters())
    for n, p in ours.named_parameters():
        print(f"grad {n:40s} ours {rel(p.grad, p64[n].grad):.4f}  autocast {rel(pbf[n].grad, p64[n].grad):.4f}")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "grads":
    grads()
