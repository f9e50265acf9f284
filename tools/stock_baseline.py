"""Stock-PyTorch (MIOpen / hipBLASLt) ResNet-34 CIFAR training step, for A/B only.

Measures what an unmodified PyTorch-ROCm training loop achieves on one MI355X so
the hand-written HIP path has a same-box comparison point.  Not the product path.
Also probes the native library interop (our ctypes kernels on torch's stream).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from kubeml_amd.models.torch_reference import resnet34


def probe_native():
    from kubeml_amd import _native
    x = torch.empty(1000, device="cuda")
    _native.HIP.call("kml_fill_f32", "p f l s", x.data_ptr(), 3.5, x.numel(), _native.stream_ptr())
    torch.cuda.synchronize()
    ok = bool((x == 3.5).all().item())
    print(json.dumps({"native_probe": ok, "abi": _native.HIP.fn("kml_abi_version", "")()}), flush=True)
    return ok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--graph", action="store_true")
    args = ap.parse_args()
    probe_native()
    torch.backends.cudnn.benchmark = True
    m = resnet34().cuda().to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(m.parameters(), lr=0.01, weight_decay=1e-4, foreach=True)
    x = torch.randn(args.batch, 3, 32, 32, device="cuda").to(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (args.batch,), device="cuda")

    def step():
        opt.zero_grad(set_to_none=False)
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            loss = F.cross_entropy(m(x), y)
        loss.backward()
        opt.step()
        return loss

    run = step
    if args.graph:
        # whole step (zero_grad, autocast forward, backward, SGD) as one captured graph:
        # stock PyTorch at its launch-overhead-free best
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                step()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        run = g.replay
    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    print(json.dumps({"stock_resnet34_bf16_autocast": True, "graph": bool(args.graph), "batch": args.batch,
                      "ms_per_step": dt * 1e3, "img_per_s": args.batch / dt}), flush=True)


if __name__ == "__main__":
    main()
