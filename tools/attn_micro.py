"""Graph-timed flash-attention kernels on the BERT-base shape (B 32, H 12, L 512, head 64):
forward, and the backward pair (dQ + dKV launched by ``attn_bwd``), with and without the
attention-probability dropout the training step uses.  One JSON line per case; the split
of the backward between its two kernels comes from a ``rocprofv3 --kernel-trace`` run of
this script.

    python tools/attn_micro.py [--B 32] [--L 512] [--H 12]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch

from kubeml_amd.ops import transformer as T
from conv_micro import gtime


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--L", type=int, default=512)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    B, H, L = a.B, a.H, a.L
    D = H * 64
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = (torch.randn(B * L, 3 * D, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    q, k, v = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
    dout = torch.randn(B * L, D, device=dev, generator=g).to(torch.bfloat16)
    dqkv = torch.empty_like(qkv)
    ctr = torch.tensor([3.0, 1.0], device=dev)
    fl_fwd = 4.0 * B * H * L * L * 64
    for name, drop in (("nodrop", None), ("drop0.1", (ctr, 77, 0.1))):
        out, lse = T.attn_fwd(q, k, v, B, H, L, drop=drop)
        tf = gtime(lambda: T.attn_fwd(q, k, v, B, H, L, out=out, drop=drop), reps=a.reps)
        tb = gtime(lambda: T.attn_bwd(q, k, v, out, dout, lse, B, H, L, dq=dqkv[:, :D], dk=dqkv[:, D:2 * D],
                                      dv=dqkv[:, 2 * D:], drop=drop), reps=a.reps)
        print(json.dumps({"case": name, "B": B, "H": H, "L": L, "fwd_us": round(tf, 2),
                          "fwd_tflops": round(fl_fwd / tf / 1e6, 1), "bwd_us": round(tb, 2),
                          "bwd_tflops": round(2.5 * fl_fwd / tb / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
