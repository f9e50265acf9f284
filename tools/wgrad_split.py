"""Split-K sweep for the hipBLASLt weight-gradient GEMM (dw[op, ip] fp32 += dy^T x, bf16 in)
on the BERT-base linear shapes (M = 32 x 512 tokens), vs the MFMA HIP wgrad kernel.
Usage: python tools/wgrad_split.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def bench(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3


def main():
    from kubeml_amd.ops import kernels as K
    dev = torch.device("cuda", 0)
    M = 16384
    for name, op, ip in [("ffn1", 3072, 768), ("ffn2", 768, 3072), ("qkv", 2304, 768), ("attn_out", 768, 768)]:
        dy = torch.randn(M, op, device=dev).bfloat16()
        x = torch.randn(M, ip, device=dev).bfloat16()
        dw = torch.zeros(op, ip, device=dev)
        fl = 2.0 * M * op * ip
        row = [f"{name:9s} op={op} ip={ip}:"]
        t = bench(lambda: K.conv_wgrad(x.view(M, 1, 1, ip), dy.view(M, 1, 1, op), dw.view(op, 1, 1, ip),
                                       1, 1, (1, 1), (0, 0)))
        row.append(f"hip {t:7.1f}us {fl / t / 1e6:6.1f}TF/s")
        for S in (1, 2, 4, 8, 16):
            if S == 1:
                f = lambda: torch.addmm(dw, dy.t(), x, out_dtype=torch.float32, out=dw)
            else:
                f = lambda S=S: dw.add_(torch.bmm(dy.view(S, M // S, op).transpose(1, 2), x.view(S, M // S, ip),
                                                  out_dtype=torch.float32).sum(0))
            t = bench(f)
            row.append(f"S={S} {t:7.1f}us {fl / t / 1e6:6.1f}")
        print(" | ".join(row), flush=True)


if __name__ == "__main__":
    main()
