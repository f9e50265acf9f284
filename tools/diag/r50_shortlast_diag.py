"""Which ResNet-50 gradients move when the 224^2 backward paths (parity-class stride-2 dgrads,
projection-shortcut dgrad last) run on a small input: ours vs fp64 / bf16-autocast per parameter."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import torch.nn.functional as F

from kubeml_amd.models import torch_reference as R
from kubeml_amd.models.resnet import resnet50
from kubeml_amd.nn import cross_entropy, flatten_module
from kubeml_amd.nn import fused
from kubeml_amd.ops import kernels as K

dev = "cuda"


def rel(a, b):
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


torch.manual_seed(0)
ref = R.resnet50(100).to(dev)
x = torch.randn(16, 3, 64, 64, device=dev).to(torch.bfloat16).float()
y = torch.randint(0, 100, (16,), device=dev)
ref64 = R.resnet50(100).to(dev).double()
ref64.load_state_dict(ref.state_dict())
ref64.train()
F.cross_entropy(ref64(x.double()), y).backward()
ac = R.resnet50(100).to(dev)
ac.load_state_dict(ref.state_dict())
ac.train()
with torch.autocast("cuda", dtype=torch.bfloat16):
    la = ac(x)
F.cross_entropy(la.float(), y).backward()
p64, pac = dict(ref64.named_parameters()), dict(ac.named_parameters())
grads = {}
for name, rows, sl in [("default", 20000, True), ("parity", 1000, False), ("parity+shortlast", 1000, True)]:
    K._S2_PARITY_MIN_ROWS = rows
    fused._SHORT_LAST = sl
    ours = resnet50(100).to(dev)
    ours.load_state_dict(ref.state_dict())
    flatten_module(ours)
    ours.train()
    cross_entropy(ours(x), y).backward()
    grads[name] = {n: p.grad.double().clone() for n, p in ours.named_parameters()}
names = [n for n in grads["default"] if "downsample" in n or "layer1.2" in n or "layer2.0" in n]
for n in names:
    g64 = p64[n].grad
    print(f"{n:40s} |g64|={g64.norm().item():.3e} ac={rel(pac[n].grad.double(), g64):.3f} " +
          " ".join(f"{k}={rel(v[n], g64):.3f}" for k, v in grads.items()) +
          f"  par-vs-def={rel(grads['parity'][n], grads['default'][n]):.3f}"
          f"  sl-vs-par={rel(grads['parity+shortlast'][n], grads['parity'][n]):.3f}", flush=True)
