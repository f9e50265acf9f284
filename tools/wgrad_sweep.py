"""Graph-timed sweep of conv weight-gradient plans (tile, split-K, variant) on ResNet-34's
3x3 / stride-1 layers at batch 256, against the tuned plan.

    python tools/wgrad_sweep.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from kubeml_amd.ops import kernels as K
from conv_micro import gtime

CFGS = [(32, 32, 64, 32, 0), (32, 32, 64, 16, 0), (64, 32, 64, 16, 0), (64, 32, 64, 8, 0), (64, 64, 64, 16, 0),
        (64, 64, 64, 8, 0), (64, 64, 64, 4, 0), (128, 64, 64, 8, 0), (64, 128, 64, 8, 0), (128, 128, 64, 4, 0),
        (64, 64, 64, 16, 1), (64, 64, 64, 8, 1), (128, 64, 64, 8, 1), (64, 128, 64, 8, 1), (128, 128, 64, 4, 1),
        (64, 64, 64, 8, 2), (128, 64, 64, 4, 2), (64, 32, 64, 16, 1), (32, 64, 64, 16, 1)]


def main():
    dev = torch.device("cuda")
    B = 256
    for (H, C, Co) in [(8, 64, 64), (4, 128, 128)]:
        x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
        dy = torch.randn(B, H, H, Co, device=dev).to(torch.bfloat16)
        dw = torch.zeros(Co, 3, 3, C, device=dev)
        ref = torch.zeros_like(dw)
        tuned = K.plan_conv("wgrad", Co, 9 * C, B * H * H)
        K.conv_wgrad(x, dy, ref, 3, 3, (1, 1), (1, 1), cfg=tuned, accumulate=False)
        res = {}
        for cfg in [tuned] + CFGS:
            try:
                K.conv_wgrad(x, dy, dw, 3, 3, (1, 1), (1, 1), cfg=cfg, accumulate=False)
                err = float((dw - ref).norm() / ref.norm())
                t = gtime(lambda: K.conv_wgrad(x, dy, dw, 3, 3, (1, 1), (1, 1), cfg=cfg, accumulate=False))
                res[str(tuple(cfg))] = (round(t, 2), round(err, 6))
            except Exception as e:  # an uninstantiated tile
                res[str(tuple(cfg))] = repr(e)[:60]
        print(json.dumps({"H": H, "C": C, "K": Co, "tuned": tuned, "us_err": res}), flush=True)


if __name__ == "__main__":
    main()
