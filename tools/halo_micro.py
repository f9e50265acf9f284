"""Graph-timed A/B of the halo-patch forward conv (variant 4) against the tuned implicit-GEMM
plan on the 3x3 / stride-1 convs of ResNet-34 (batch 256): every instantiated halo tile,
with the BN partial-statistics epilogue the training step uses.

    python tools/halo_micro.py [--batch 256]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from kubeml_amd.ops import kernels as K
from conv_micro import gtime


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--oneshot", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda")
    B = a.batch
    for (H, C, Co) in [(8, 64, 64), (4, 128, 128), (8, 256, 256), (4, 512, 512)]:
        x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(Co, 3, 3, C, device=dev) * 0.05).to(torch.bfloat16)
        y = torch.empty(B, H, H, Co, dtype=torch.bfloat16, device=dev)
        M, Kd = B * H * H, 9 * C
        base = K.plan_conv("fwd", M, Co, Kd)
        rows = {}
        for cfg in [base] + [(bm, bn, 0, 1, K.HALO) for bm, bn in K._HALO_TILES[(C, H)] if Co % bn == 0]:
            G = K.conv_fwd_stats_rows(x.shape, Co, 3, 3, (1, 1), (1, 1), cfg=cfg)
            st = torch.empty(G * 2 * Co, device=dev)
            t = gtime(lambda: K.conv_fwd(x, w, 3, 3, (1, 1), (1, 1), out=y, stats=st, stats_part=True, cfg=cfg))
            rows[str(tuple(cfg))] = round(t, 2)
        fl = 2 * M * Co * Kd
        best = min(rows.values())
        print(json.dumps({"H": H, "C": C, "K": Co, "M": M, "us": rows, "best_tflops": round(fl / best / 1e6, 1)}),
              flush=True)




def oneshot_main():
    """One-shot panel kernel (variant 5) vs the tuned plan: layer3's unrolled 2x2 convs
    (1x1 form, weight gathered from the 3x3 weight) and layer4's centre-tap convs."""
    dev = torch.device("cuda")
    B = 256
    for name, (H, C, Co, unroll) in {"layer3_unrolled": (2, 256, 256, True), "layer4": (1, 512, 512, False)}.items():
        x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(Co, 3, 3, C, device=dev) * 0.05).to(torch.bfloat16)
        M, N, Kd = (B, 4 * Co, 4 * C) if unroll else (B, Co, C)
        base = K.plan_conv("fwd", M, N, Kd)
        rows = {}
        for cfg in [base] + [(bm, bn, 0, 1, K.ONESHOT) for bm, bn in K._ONESHOT_TILES[Kd]]:
            G = K.conv_fwd_stats_rows(x.shape, Co, 3, 3, (1, 1), (1, 1), cfg=cfg, unroll=unroll)
            st = torch.empty(G * 2 * Co, device=dev)
            kw = dict(wu=K.GATHER22) if unroll else {}
            t = gtime(lambda: K.conv_fwd(x, w, 3, 3, (1, 1), (1, 1), stats=st, stats_part=True, cfg=cfg, **kw))
            rows[str(tuple(cfg))] = round(t, 2)
        print(json.dumps({"layer": name, "M": M, "N": N, "K": Kd, "us": rows}), flush=True)


if __name__ == "__main__":
    if "--oneshot" in sys.argv:
        oneshot_main()
    else:
        main()
