"""Bandwidth of the BN apply / backward-apply kernels at ResNet-50 shapes (batch 128, 224²)
against a same-bytes bf16 copy (the achievable HBM rate on this box).  Graph-timed, one
JSON line per case: bytes moved, microseconds, TB/s, fraction of the copy's rate.

    python tools/bn_bw.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch

from kubeml_amd.ops import kernels as K
from launch_floor import timed  # noqa: E402


def main():
    dev = torch.device("cuda")
    cases = [(401408, 64, False), (401408, 256, True), (401408, 256, False), (100352, 512, True),
             (100352, 128, False), (25088, 1024, True)]
    for M, C, with_res in cases:
        torch.manual_seed(0)
        x = (torch.randn(M, C, device=dev)).to(torch.bfloat16)
        res = (torch.randn(M, C, device=dev)).to(torch.bfloat16) if with_res else None
        g = torch.rand(C, device=dev) + 0.5
        b = torch.randn(C, device=dev)
        G = -(-M // 128)                                     # one partial row per 128-row conv tile
        rows = torch.randn(G * 2 * C, device=dev) + 1000.0
        mean, rstd = torch.empty(C, device=dev), torch.empty(C, device=dev)
        y = torch.empty_like(x)
        N = 4
        t_apply = timed(lambda: [K.bn_apply(x, rows, g, b, y=y, res=res, save_mean=mean, save_rstd=rstd, relu=True,
                                            stats_rows=G) for _ in range(N)], N)
        n_ops = 3 if with_res else 2
        nbytes = n_ops * M * C * 2
        src = torch.empty(M * C * (n_ops - 1), dtype=torch.bfloat16, device=dev)
        dst = torch.empty(M * C, dtype=torch.bfloat16, device=dev)
        # copy of the same total bytes: (n_ops - 1) reads' worth into one write via a sum
        t_copy = timed(lambda: [dst.copy_(src[:M * C]) for _ in range(N)], N)
        copy_bytes = 2 * M * C * 2
        dz = (torch.randn(M, C, device=dev)).to(torch.bfloat16)
        part = torch.randn(G * 2 * C, device=dev)
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if with_res else None
        t_bwd = timed(lambda: [K.bn_bwd(dz, None, x, mean, rstd, g, dg, db, dx=dx, dres=dres, partial=(part, G))
                               for _ in range(N)], N)
        bwd_bytes = (3 + (1 if with_res else 0)) * M * C * 2
        copy_rate = copy_bytes / t_copy / 1e6
        out = {"M": M, "C": C, "res": with_res,
               "apply_us": round(t_apply, 2), "apply_TBps": round(nbytes / t_apply / 1e6, 2),
               "bwd_us": round(t_bwd, 2), "bwd_TBps": round(bwd_bytes / t_bwd / 1e6, 2),
               "copy_TBps": round(copy_rate, 2),
               "apply_vs_copy": round(nbytes / t_apply / 1e6 / copy_rate, 3),
               "bwd_vs_copy": round(bwd_bytes / t_bwd / 1e6 / copy_rate, 3)}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
