"""Per-call timing of the conv / BN kernels of one eager ResNet training step.

Wraps the ``ops.kernels`` entry points the fused modules call, synchronises around each
call and prints one line per call (entry point, shapes, plan, flags, microseconds), then a
table of the slowest calls.  Eager timing includes per-call sync overhead (a few us): use
it to find WHICH call is slow and with which operand shapes, then look the kernel up in a
rocprofv3 trace of the graphed step.

    python tools/conv_calls.py [--model resnet50|vgg16] [--batch 128] [--size 224] [--top 30]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--size", type=int, default=224)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    from kubeml_amd.models import resnet as R
    from kubeml_amd.models import vgg as VG
    from kubeml_amd.nn import backward_loss, cross_entropy, flatten_module
    from kubeml_amd.ops import kernels as K

    dev = torch.device("cuda")
    torch.manual_seed(0)
    if a.model.startswith("vgg"):
        model = getattr(VG, a.model)(100).to(dev)     # VGG-16-BN / CIFAR-100 (config 4)
    else:
        model = getattr(R, a.model)(1000 if a.size > 64 else 10).to(dev)
    flatten_module(model)
    model.train()
    x = (torch.randn(a.batch, a.size, a.size, 8, device=dev) * 0.5).to(torch.bfloat16)
    x[..., 3:] = 0
    y = torch.randint(0, 100 if a.model.startswith("vgg") else (1000 if a.size > 64 else 10), (a.batch,), device=dev)

    calls = []
    active = [False]

    def desc(v):
        if isinstance(v, torch.Tensor):
            return list(v.shape)
        if isinstance(v, (tuple, list)) and v and all(isinstance(e, torch.Tensor) or e is None for e in v):
            return [desc(e) for e in v]
        if isinstance(v, (int, float, str, bool, type(None))):
            return v
        if isinstance(v, (tuple, list)):
            return [desc(e) for e in v]
        return type(v).__name__

    def wrap(name):
        fn = getattr(K, name)

        def w(*args, **kw):
            if not active[0]:
                return fn(*args, **kw)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = fn(*args, **kw)
            torch.cuda.synchronize()
            us = (time.perf_counter() - t0) * 1e6
            info = {"fn": name, "us": round(us, 1), "args": [desc(v) for v in args[:4]],
                    "kw": {k: desc(v) for k, v in kw.items() if v is not None and k not in ("out",)}}
            if name in ("conv_bwd",):
                xs = args[2].shape
                info["plans"] = [list(p) if isinstance(p, tuple) else p
                                 for p in K.bwd_plans(tuple(xs), args[1].shape[0], args[4], args[5], args[6], args[7],
                                                      kw.get("dcfg"), kw.get("wcfg"))]
            calls.append(info)
            return r
        setattr(K, name, w)

    for n in ("conv_fwd", "conv_dgrad", "conv_wgrad", "conv_bwd", "conv_fwd_bnin", "bn_apply", "bn_bwd",
              "bn_relu_maxpool", "maxpool_bwd", "fold22_multi", "sgd_"):
        if hasattr(K, n):
            wrap(n)

    def step():
        loss = cross_entropy(model(x), y)
        backward_loss(loss)
        return loss

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    active[0] = True
    t0 = time.perf_counter()
    step()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    active[0] = False
    for c in calls:
        print(json.dumps(c))
    tot = sum(c["us"] for c in calls)
    print(f"# {len(calls)} calls, {tot / 1e3:.2f} ms in wrapped calls, step wall {wall:.2f} ms (eager, synced)")
    for c in sorted(calls, key=lambda c: -c["us"])[:a.top]:
        print(f"# {c['us']:9.1f}  {c['fn']:14s} {c['args']} {c.get('plans', '')} {sorted(c['kw'])}")


if __name__ == "__main__":
    main()
