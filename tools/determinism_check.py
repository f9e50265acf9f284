"""Run the same KubeModel training (ResNet-18, batches 32/32/20/32/32, reset at 3) several
times from one init on the graphed and eager paths and report per-run update norms and
pairwise differences — tells run-to-run nondeterminism (atomic order) from a path bug."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

dev = torch.device("cuda", 0)


def main():
    from kubeml_amd.models.resnet import resnet18
    from kubeml_amd.nn import flatten_module
    from kubeml_amd.optim import SGD
    from kubeml_amd.sdk.model import KubeModel
    g = torch.Generator(device=dev).manual_seed(7)
    data = []
    for b in [32, 32, 20, 32, 32]:
        x = torch.randn(b, 32, 32, 8, device=dev, generator=g).to(torch.bfloat16)
        x[..., 3:] = 0
        data.append((x, torch.randint(0, 10, (b,), device=dev, generator=g)))
    # poison the caching allocator: blocks handed out later start as NaN, so a kernel that
    # reads memory nobody wrote shows up as a NaN loss instead of a rare divergence
    if os.environ.get("POISON", "1") == "1":
        junk = [torch.full((1 << 26,), float("nan"), device=dev) for _ in range(16)]
        small = [torch.full((n,), float("nan"), device=dev) for n in (1 << 10, 1 << 12, 1 << 14, 1 << 16, 1 << 18)
                 for _ in range(64)]
        del junk, small
    torch.manual_seed(0)
    ref = resnet18(10)
    sd = {k: v.clone() for k, v in ref.state_dict().items()}
    ups = []
    for run in range(int(os.environ.get("RUNS", "6"))):
        graph = run % 2 == 0
        os.environ.pop("KUBEML_NO_GRAPH", None) if graph else os.environ.__setitem__("KUBEML_NO_GRAPH", "1")
        net = resnet18(10)
        net.load_state_dict(sd)

        class M(KubeModel):
            pass
        km = M(net, None, gpu=True)
        net.to(dev)
        km.device = dev
        km._flat = flatten_module(net)
        km.optimizer = SGD(net.parameters(), lr=1e-3, momentum=0.9, dampening=0.1, weight_decay=1e-4)
        w0 = km._flat.master.clone()
        losses = []
        for i, (x, y) in enumerate(data):
            if i == 3:
                km.optimizer.reset_state()
            losses.append(round(float(km.step(x, y).detach()), 6))
        torch.cuda.synchronize()
        u = km._flat.master - w0
        ups.append(u)
        print("run", run, "graph" if graph else "eager", losses, "upd_norm %.6g" % float(u.norm()), flush=True)
    for i in range(len(ups)):
        print(i, ["%.3g" % float((ups[i] - ups[j]).norm() / ups[j].norm()) for j in range(len(ups))])


if __name__ == "__main__":
    main()
