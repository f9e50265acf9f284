"""VGG-16-BN / CIFAR-100 training throughput on one MI355X (north-star config 4's model).

The graphed train step of the framework (engine/dp.py make_train_step: forward, loss,
backward, fused Adam, one hipGraph replay) on synthetic CIFAR-100-shaped uint8 images resident
in HBM with the on-device crop/flip/normalise kernel; random-init weights.  The reference's VGG
function trained with Adam (ml/experiments/kubeml/function_vgg11.py:54).

    python tools/bench_vgg.py [--batch 128] [--steps 50] [--warmup 5] [--opt adam|sgd]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--images", type=int, default=50000)
    ap.add_argument("--opt", choices=["adam", "sgd"], default="adam")
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--opt-overlap", choices=["on", "off"], default="off",
                    help="per-stage optimizer on a side stream (classifier update beside the conv backward)")
    a = ap.parse_args()
    import torch
    from kubeml_amd.engine.dp import make_train_step
    from kubeml_amd.models.vgg import vgg16
    from kubeml_amd.nn import cross_entropy, flatten_module
    from kubeml_amd.ops import kernels as K
    from kubeml_amd.optim import SGD, Adam
    dev = torch.device("cuda", 0)
    B = a.batch
    g = torch.Generator(device=dev).manual_seed(0)
    data = torch.randint(0, 256, (a.images, 32, 32, 3), dtype=torch.uint8, device=dev, generator=g)
    labels = torch.randint(0, 100, (a.images,), dtype=torch.int64, device=dev, generator=g)
    ctr = torch.tensor([5.0, 0.0, 0.0], dtype=torch.float32, device=dev)
    xbuf = torch.empty((B, 32, 32, 8), dtype=torch.bfloat16, device=dev)
    ybuf = torch.empty((B,), dtype=torch.int64, device=dev)
    torch.manual_seed(0)
    model = vgg16(100).to(dev)
    space = flatten_module(model)
    model.train()
    opt = Adam(model.parameters(), lr=a.lr) if a.opt == "adam" else SGD(model.parameters(), lr=a.lr, momentum=0.9,
                                                                         weight_decay=5e-4)
    step = make_train_step(model, space, opt, cross_entropy, xbuf, ybuf,
                           pre=lambda: K.augment(data, labels, ctr, B, out=xbuf, labels_out=ybuf, train=True),
                           advance=(ctr, B, a.images), extra_state=[ctr], opt_overlap=a.opt_overlap == "on")
    step.capture()
    for _ in range(a.warmup):
        loss = step()
    torch.cuda.synchronize()
    l0 = float(loss)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ms = dt / a.steps * 1e3
    print(json.dumps({"metric": "VGG-16-BN CIFAR-100 training images/s (1 GPU, graphed step)",
                      "value": round(B * a.steps / dt, 1), "unit": "images/s", "ms_per_step": round(ms, 4),
                      "batch": B, "optimizer": a.opt, "steps": a.steps, "warmup": a.warmup,
                      "opt_overlap": bool(getattr(step, "segment_opt", None)),
                      "loss_first_last": [round(l0, 4), round(float(loss), 4)],
                      "data": "synthetic CIFAR-100-shaped uint8 in HBM, on-device crop/flip/normalise; random init"}),
          flush=True)


if __name__ == "__main__":
    main()
