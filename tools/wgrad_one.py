"""One ResNet-50 1x1 weight-gradient shape, one route, a few reps (for rocprofv3 --pmc passes).

    python tools/wgrad_one.py --P 401408 --K 128 --C 256 --route conv|slab [--reps 5]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from kubeml_amd.ops import gemm as G
from kubeml_amd.ops import kernels as K


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=401408)
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--C", type=int, default=256)
    ap.add_argument("--route", default="slab")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    B = 128
    hw = int(round((a.P // B) ** 0.5))
    x = torch.randn(B, hw, hw, a.C, device=dev).to(torch.bfloat16)
    dy = torch.randn(B, hw, hw, a.K, device=dev).to(torch.bfloat16)
    dw = torch.zeros(a.K, 1, 1, a.C, device=dev)
    route = K.wgrad_gemm_route(x.shape, a.K, 1, 1, (1, 1), (0, 0))
    for _ in range(a.reps):
        if a.route == "conv":
            K.conv_wgrad(x, dy, dw, 1, 1, (1, 1), (0, 0), cfg=K.plan_conv("wgrad", a.K, a.C, a.P), accumulate=False)
        else:
            _, bm, bn, st, sp = route
            G.wgrad_splitk_(dw.view(a.K, a.C), dy.view(-1, a.K), a.K, x.view(-1, a.C), a.C, a.K, a.C, a.P, beta=0.0,
                            tile=(bm, bn, st) if st else (bm, bn), splits=sp)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
