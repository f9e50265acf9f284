"""Where does a ResNet-34 BN apply's time go?  Graph-timed, per launch, at the batch-256
shapes: the launch floor (tiny kernel), a same-size streaming relu (bytes floor),
bn_apply from final [2C] sums (stats_rows=0) and from G per-wave partial rows (the conv
epilogue's layout) for several G; plus the backward apply with partial rows."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kubeml_amd.ops import kernels as K  # noqa: E402
from launch_floor import timed  # noqa: E402


def main():
    dev = torch.device("cuda")
    N = 50
    ctr = torch.zeros(3, device=dev)
    print("tiny kernel us %.2f" % timed(lambda: [K.advance_counter_(ctr, 256, 50000) for _ in range(N)], N))
    for M, C in ((65536, 64), (16384, 64), (4096, 128), (1024, 256), (256, 512)):
        x = torch.randn(M, C, device=dev).to(torch.bfloat16)
        g = torch.rand(C, device=dev) + 0.5
        b = torch.randn(C, device=dev)
        mean, rstd = torch.empty(C, device=dev), torch.empty(C, device=dev)
        st = torch.zeros(2 * C, device=dev)
        K.bn_stats(x, st)
        row = {"M": M, "C": C}
        row["relu_us"] = timed(lambda: [K.relu_fwd(x) for _ in range(N)], N)
        row["apply_final_us"] = timed(lambda: [K.bn_apply(x, st, g, b, save_mean=mean, save_rstd=rstd, relu=True)
                                               for _ in range(N)], N)
        for G in (1, 8, 32, 128, 512):
            part = (st / G).repeat(G)
            row[f"apply_G{G}_us"] = timed(lambda: [K.bn_apply(x, part, g, b, save_mean=mean, save_rstd=rstd, relu=True,
                                                              stats_rows=G) for _ in range(N)], N)
        print({k: (round(v, 2) if isinstance(v, float) else v) for k, v in row.items()}, flush=True)


if __name__ == "__main__":
    main()
