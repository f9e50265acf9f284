"""Diagnostic: KubeModel.step graph path vs eager path vs eager path (determinism)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_engine_gpu import _batches, _km  # noqa: E402

from kubeml_amd.models.resnet import resnet18  # noqa: E402
from kubeml_amd.optim import SGD  # noqa: E402

mom = float(sys.argv[1]) if len(sys.argv) > 1 else 0.9


def opt(ps):
    return SGD(ps, lr=0.05, momentum=mom, dampening=0.1 if mom else 0.0, weight_decay=1e-4)


torch.manual_seed(0)
nets = [resnet18(10) for _ in range(3)]
for n in nets[1:]:
    n.load_state_dict(nets[0].state_dict())
kms = [_km(n, opt) for n in nets]
data = _batches()
modes = ["graph", "eager", "eager"]
for i, (x, y) in enumerate(data):
    losses = []
    for km, m in zip(kms, modes):
        if m == "graph":
            os.environ.pop("KUBEML_NO_GRAPH", None)
        else:
            os.environ["KUBEML_NO_GRAPH"] = "1"
        losses.append(float(km.step(x, y)))
    torch.cuda.synchronize()
    ms = [k._flat.master for k in kms]
    gs = [k._flat.grad for k in kms]
    print(f"step {i} losses {losses}  |m_g-m_e| {float((ms[0]-ms[1]).abs().max()):.3e} "
          f"|m_e-m_e| {float((ms[1]-ms[2]).abs().max()):.3e}  |g_g-g_e| {float((gs[0]-gs[1]).abs().max()):.3e} "
          f"|g_e-g_e| {float((gs[1]-gs[2]).abs().max()):.3e} gmax {float(gs[1].abs().max()):.3e}", flush=True)
