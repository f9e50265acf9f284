"""Graph-timed microbenchmarks of single conv launches vs library references.

For a few ResNet-34/CIFAR layers (batch 256): our fwd conv with/without the BN-stats
epilogue, and torch (hipBLASLt GEMM of the same implicit-GEMM shape, MIOpen conv).
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from kubeml_amd.ops import kernels as K


def gtime(fn, reps=50):
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        for _ in range(2):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(st):
        with torch.cuda.graph(g, stream=st):
            for _ in range(reps):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / 5 / reps * 1e6


def main():
    dev = torch.device("cuda")
    layers = [  # B, H, W, Ci, Co, k, s, p
        (256, 8, 8, 64, 64, 3, 1, 1),
        (256, 4, 4, 128, 128, 3, 1, 1),
        (256, 2, 2, 256, 256, 3, 1, 1),
        (256, 1, 1, 512, 512, 3, 1, 1),
    ]
    for (B, H, W, Ci, Co, k, s, p) in layers:
        x = torch.randn(B, H, W, Ci, device=dev).to(torch.bfloat16)
        w = (torch.randn(Co, k, k, Ci, device=dev) * 0.05).to(torch.bfloat16)
        OH, OW = K.out_hw(H, W, k, k, s, s, p, p)
        y = torch.empty(B, OH, OW, Co, dtype=torch.bfloat16, device=dev)
        stats = torch.zeros(2 * Co, device=dev)
        M, N, Kd = B * OH * OW, Co, k * k * Ci
        cfg = K.plan_conv("fwd", M, N, Kd)
        t_ns = gtime(lambda: K.conv_fwd(x, w, k, k, (s, s), (p, p), out=y))
        t_st = gtime(lambda: K.conv_fwd(x, w, k, k, (s, s), (p, p), out=y, stats=stats))
        A = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
        Bm = torch.randn(Kd, N, device=dev).to(torch.bfloat16)
        C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        t_mm = gtime(lambda: torch.mm(A, Bm, out=C))
        xc = x.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        wc = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        t_cv = gtime(lambda: F.conv2d(xc, wc, stride=s, padding=p))
        fl = 2 * M * N * Kd
        print(f"M={M} N={N} K={Kd} cfg={cfg}: ours {t_ns:.2f}us (+stats {t_st:.2f}us) "
              f"[{fl / t_ns / 1e6:.1f} TF/s]  hipblaslt-mm {t_mm:.2f}us  miopen {t_cv:.2f}us", flush=True)


if __name__ == "__main__":
    main()
