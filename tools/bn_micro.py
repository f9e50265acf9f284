"""Graph-timed BN kernels at the ResNet-34 / batch-256 shapes (bn_apply, bn_bwd in both
reduce modes) — per-launch device time without profiler overhead."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from kubeml_amd.ops import kernels as K
from launch_floor import timed  # noqa: E402


def main():
    dev = torch.device("cuda")
    for M, C in ((65536, 64), (16384, 64), (4096, 128), (1024, 256), (256, 512)):
        x = torch.randn(M, C, device=dev).to(torch.bfloat16)
        dy = torch.randn(M, C, device=dev).to(torch.bfloat16)
        g = torch.rand(C, device=dev) + 0.5
        b = torch.randn(C, device=dev)
        st = torch.zeros(2 * C, device=dev)
        K.bn_stats(x, st)
        mean, rstd = torch.empty(C, device=dev), torch.empty(C, device=dev)
        y = K.bn_apply(x, st, g, b, save_mean=mean, save_rstd=rstd, relu=True)
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        N = 20
        t_apply = timed(lambda: [K.bn_apply(x, st, g, b, save_mean=mean, save_rstd=rstd, relu=True)
                                 for _ in range(N)], N)
        res = {}
        for mode in ("fused", "ticket", "atomic"):
            K._BN_REDUCE = mode
            res[mode] = timed(lambda: [K.bn_bwd(dy, y, x, mean, rstd, g, dg, db) for _ in range(N)], N)
        print(f"M={M} C={C}: bn_apply {t_apply:.2f} us  bn_bwd " +
              "  ".join(f"{k} {v:.2f} us" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
