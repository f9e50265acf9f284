"""Training-stability probe: loss per step for eager vs graphed ResNet-34 steps."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from kubeml_amd.engine.step import GraphedTrainStep
from kubeml_amd.models.resnet import resnet34
from kubeml_amd.nn import cross_entropy, flatten_module
from kubeml_amd.ops import kernels as K
from kubeml_amd.optim import SGD


def run(graph, steps=12, B=256, lr=0.01, N=4096, warmup=2, seed=0, datafirst=0, setdev=0, nosync=0, bigalloc=0):
    dev = torch.device("cuda")
    if setdev:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
    if datafirst:
        g = torch.Generator(device=dev).manual_seed(0)
        data = torch.randint(0, 256, (N, 32, 32, 3), dtype=torch.uint8, device=dev, generator=g)
        labels = torch.randint(0, 10, (N,), device=dev, generator=g)
    torch.manual_seed(seed)
    model = resnet34(1000).to(dev)
    space = flatten_module(model)
    opt = SGD(model.parameters(), lr=lr, weight_decay=1e-4)
    if not datafirst:
        g = torch.Generator(device=dev).manual_seed(0)
        data = torch.randint(0, 256, (N, 32, 32, 3), dtype=torch.uint8, device=dev, generator=g)
        labels = torch.randint(0, 10, (N,), device=dev, generator=g)
    ctr = torch.tensor([1.0, 0.0, 0.0], device=dev)
    xb = torch.empty(B, 32, 32, 8, dtype=torch.bfloat16, device=dev)
    yb = torch.empty(B, dtype=torch.int64, device=dev)

    def fb():
        K.augment(data, labels, ctr, B, out=xb, labels_out=yb, train=True)
        space.zero_grad()
        loss = cross_entropy(model(xb), yb)
        loss.backward()
        return loss

    def os_():
        opt.step()
        K.advance_counter_(ctr, B, N)

    st = GraphedTrainStep(fb, os_, use_graph=graph, warmup=warmup)
    st.capture()
    out = []
    for i in range(steps):
        for _ in range(nosync):
            st()
        l = st()
        if bigalloc:
            junk = torch.full((int(bigalloc) * 2**20,), float("inf"), device=dev)
            del junk
        out.append(round(float(l.item()), 3))
        gn = float(space.grad.norm().item())
        if i < 3 or i % 5 == 0:
            print(f"  step {i} loss {out[-1]} gradnorm {gn:.3e} wnorm {float(space.master.norm()):.3e}", flush=True)
    return out


if __name__ == "__main__":
    mode = sys.argv[1] if len(sys.argv) > 1 else "both"
    if mode == "both":
        for graph in (False, True):
            print("graph" if graph else "eager", flush=True)
            print(run(graph), flush=True)
    else:
        kw = dict(a.split("=") for a in sys.argv[2:])
        kw = {k: int(v) for k, v in kw.items()}
        print(mode, kw, flush=True)
        print(run(mode == "graph", **kw), flush=True)
