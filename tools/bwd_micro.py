"""Graph-timed split of a conv backward on ResNet-34's 3x3 / stride-1 layers (batch 256):
the grouped dgrad+wgrad launch the step uses (``conv_bwd``), and dgrad / wgrad alone with
the same plans.

    python tools/bwd_micro.py [--batch 256]
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
    a = ap.parse_args()
    dev = torch.device("cuda")
    B = a.batch
    for (H, C, Co) in [(8, 64, 64), (4, 128, 128)]:
        x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(Co, 3, 3, C, device=dev) * 0.05).to(torch.bfloat16)
        dy = torch.randn(B, H, H, Co, device=dev).to(torch.bfloat16)
        dw = torch.zeros(Co, 3, 3, C, device=dev)
        dplan, wplan, grouped = K.bwd_plans(x.shape, Co, 3, 3, (1, 1), (1, 1))
        r = {"dplan": dplan, "wplan": wplan, "grouped": grouped}
        M = B * H * H
        base = K.plan_conv("dgrad", M, C, 9 * Co)
        r["base_dplan"] = base
        r["bwd_us"] = round(gtime(lambda: K.conv_bwd(dy, w, x, dw, 3, 3, (1, 1), (1, 1), accumulate=False)), 2)
        r["pair_base_us"] = round(gtime(lambda: K.conv_bwd(dy, w, x, dw, 3, 3, (1, 1), (1, 1), accumulate=False,
                                                           dcfg=base, wcfg=wplan)), 2)
        r["dgrad_us"] = round(gtime(lambda: K.conv_dgrad(dy, w, x.shape, 3, 3, (1, 1), (1, 1), cfg=dplan)), 2)
        r["dgrad_base_us"] = round(gtime(lambda: K.conv_dgrad(dy, w, x.shape, 3, 3, (1, 1), (1, 1), cfg=base)), 2)
        r["wgrad_us"] = round(gtime(lambda: K.conv_wgrad(x, dy, dw, 3, 3, (1, 1), (1, 1), cfg=wplan,
                                                         accumulate=False)), 2)
        r["gflop_each"] = round(2 * M * Co * 9 * C / 1e9, 3)
        print(json.dumps({"H": H, "C": C, "K": Co, **r}), flush=True)


if __name__ == "__main__":
    main()
