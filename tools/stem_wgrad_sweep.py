"""Graph-timed sweep of the stem's weight-gradient plan (7x7/s2, Cin 8, Cout 64, batch 256):
M = 64, N = 392, K = 65536 pixels — a long-K GEMM with a tiny output, i.e. all split-K."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from kubeml_amd.ops import kernels as K
from conv_micro import gtime


def main():
    dev = torch.device("cuda")
    B = 256
    x = torch.randn(B, 32, 32, 8, device=dev).to(torch.bfloat16)
    dy = torch.randn(B, 16, 16, 64, device=dev).to(torch.bfloat16)
    dw = torch.zeros(64, 7, 7, 8, device=dev)
    ref = torch.zeros_like(dw)
    cur = K.plan_conv("wgrad", 64, 392, 65536)
    K.conv_wgrad(x, dy, ref, 7, 7, (2, 2), (3, 3), cfg=cur, accumulate=False)
    res = {}
    cands = [cur] + [(bm, bn, 64, sp, v) for (bm, bn) in ((64, 32), (64, 64), (64, 128), (32, 64), (32, 32))
                     for sp in (32, 64, 128, 256) for v in (0, 1)]
    for cfg in cands:
        try:
            K.conv_wgrad(x, dy, dw, 7, 7, (2, 2), (3, 3), cfg=cfg, accumulate=False)
            err = float((dw - ref).norm() / ref.norm())
            t = gtime(lambda: K.conv_wgrad(x, dy, dw, 7, 7, (2, 2), (3, 3), cfg=cfg, accumulate=False))
            res[str(tuple(cfg))] = (round(t, 2), round(err, 6))
        except Exception as e:
            res[str(tuple(cfg))] = repr(e)[:50]
    best = sorted((v[0], k) for k, v in res.items() if isinstance(v, tuple))[:5]
    print(json.dumps({"current": cur, "best5": best, "all": res}), flush=True)


if __name__ == "__main__":
    main()
