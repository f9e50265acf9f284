"""ResNet-34 / CIFAR backward pairs, layer by layer: the shipped plans vs alternative weight-
gradient plans (tile x split-K), alone and inside the grouped dgrad+wgrad launch.  Graph-timed
(tools/conv_micro.gtime), batch 256, 3x3 stride-1 convs of layers 1-4.

    python tools/wgrad_sweep_r34.py [--batch 256]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from kubeml_amd.ops import kernels as K  # noqa: E402
from conv_micro import gtime  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    dev = torch.device("cuda")
    B = a.batch
    for (H, C) in [(8, 64), (4, 128), (2, 256), (1, 512)]:
        x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(C, 3, 3, C, device=dev) * 0.05).to(torch.bfloat16)
        dy = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
        dw = torch.zeros(C, 3, 3, C, device=dev)
        dplan, wplan, grouped = K.bwd_plans(x.shape, C, 3, 3, (1, 1), (1, 1))
        base = {"H": H, "C": C, "dplan": list(dplan), "wplan": list(wplan), "grouped": grouped}
        base["pair_us"] = round(gtime(lambda: K.conv_bwd(dy, w, x, dw, 3, 3, (1, 1), (1, 1), accumulate=False)), 2)
        base["dgrad_us"] = round(gtime(lambda: K.conv_dgrad(dy, w, x.shape, 3, 3, (1, 1), (1, 1), cfg=dplan)), 2)
        base["wgrad_us"] = round(gtime(lambda: K.conv_wgrad(x, dy, dw, 3, 3, (1, 1), (1, 1), cfg=wplan,
                                                            accumulate=False)), 2)
        print(json.dumps(base), flush=True)
        ref = dw.clone()
        for bm, bn in ((32, 32), (64, 32)):
            for s in (2, 4, 8, 16, 32, 64):
                cfg = (bm, bn, 64, s, 0)
                try:
                    tw = gtime(lambda: K.conv_wgrad(x, dy, dw, 3, 3, (1, 1), (1, 1), cfg=cfg, accumulate=False))
                    ok = bool(torch.allclose(dw, ref, rtol=1e-4, atol=1e-3))
                    tp = gtime(lambda: K.conv_bwd(dy, w, x, dw, 3, 3, (1, 1), (1, 1), accumulate=False, dcfg=dplan,
                                                  wcfg=cfg))
                except Exception as e:  # a plan the launcher rejects
                    print(json.dumps({"H": H, "C": C, "wcfg": list(cfg), "error": repr(e)[:120]}), flush=True)
                    continue
                print(json.dumps({"H": H, "C": C, "wcfg": list(cfg), "wgrad_us": round(tw, 2), "pair_us": round(tp, 2),
                                  "matches_shipped": ok}), flush=True)


if __name__ == "__main__":
    main()
