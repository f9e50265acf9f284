"""Graph-timed GEMM/conv microbenchmark on the large shapes (BERT-base linears, ResNet-50
ImageNet convs): our MFMA kernels vs hipBLASLt (torch.mm) and MIOpen (F.conv2d).

Usage: python tools/gemm_micro.py [--bert] [--r50]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from kubeml_amd.ops import kernels as K
from conv_micro import gtime  # noqa: E402


def bert(dev, T=8192):
    # (name, M, N, K): y[M,N] = x[M,K] @ W[N,K]^T   (nn.Linear), T tokens
    shapes = [("qkv", T, 2304, 768), ("attn_out", T, 768, 768), ("ffn1", T, 3072, 768), ("ffn2", T, 768, 3072)]
    for name, M, N, Kd in shapes:
        x = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, Kd, device=dev) * 0.05).to(torch.bfloat16)
        x4 = x.view(M, 1, 1, Kd)
        w4 = w.view(N, 1, 1, Kd)
        y = torch.empty(M, 1, 1, N, dtype=torch.bfloat16, device=dev)
        t_ours = gtime(lambda: K.conv_fwd(x4, w4, 1, 1, (1, 1), (0, 0), out=y), reps=20)
        wt = w.t().contiguous()
        yc = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        t_mm = gtime(lambda: torch.mm(x, wt, out=yc), reps=20)
        t_lin = gtime(lambda: F.linear(x, w), reps=20)
        fl = 2 * M * N * Kd
        print(f"bert {name:9s} M={M} N={N} K={Kd}: ours {t_ours:8.2f}us {fl / t_ours / 1e6:6.1f} TF/s | "
              f"hipblaslt mm {t_mm:8.2f}us {fl / t_mm / 1e6:6.1f} TF/s | linear {t_lin:8.2f}us", flush=True)
        ref = F.linear(x.float(), w.float())
        K.conv_fwd(x4, w4, 1, 1, (1, 1), (0, 0), out=y)
        err = (y.view(M, N).float() - ref).abs().max().item() / ref.abs().max().item()
        print(f"   rel max err {err:.2e}")


def r50(dev, B=64):
    layers = [  # H, W, Ci, Co, k, s, p
        (56, 56, 64, 64, 1, 1, 0), (56, 56, 64, 64, 3, 1, 1), (56, 56, 64, 256, 1, 1, 0),
        (28, 28, 128, 128, 3, 1, 1), (28, 28, 512, 128, 1, 1, 0), (14, 14, 256, 256, 3, 1, 1),
        (14, 14, 1024, 256, 1, 1, 0), (7, 7, 512, 512, 3, 1, 1), (7, 7, 2048, 512, 1, 1, 0),
    ]
    for (H, W, Ci, Co, k, s, p) in layers:
        x = torch.randn(B, H, W, Ci, device=dev).to(torch.bfloat16)
        w = (torch.randn(Co, k, k, Ci, device=dev) * 0.05).to(torch.bfloat16)
        OH, OW = K.out_hw(H, W, k, k, s, s, p, p)
        y = torch.empty(B, OH, OW, Co, dtype=torch.bfloat16, device=dev)
        M, N, Kd = B * OH * OW, Co, k * k * Ci
        t_ours = gtime(lambda: K.conv_fwd(x, w, k, k, (s, s), (p, p), out=y), reps=20)
        xc = x.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        wc = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        t_cv = gtime(lambda: F.conv2d(xc, wc, stride=s, padding=p), reps=20)
        fl = 2 * M * N * Kd
        print(f"r50 {H}x{W} {Ci}->{Co} k{k}: M={M} N={N} K={Kd}: ours {t_ours:8.2f}us {fl / t_ours / 1e6:6.1f} TF/s"
              f" | miopen {t_cv:8.2f}us {fl / t_cv / 1e6:6.1f} TF/s", flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--bert", action="store_true")
    ap.add_argument("--r50", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda")
    if a.bert or not a.r50:
        bert(dev)
    if a.r50 or not a.bert:
        r50(dev)
