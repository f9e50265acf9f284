"""Print graph-timed us for every (tile, bk, variant, splits) of ONE conv shape.

    python tools/conv_sweep.py --mode fwd --B 256 --H 2 --W 2 --cin 256 --cout 256 --k 3 --s 1 --p 1
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from kubeml_amd.ops import kernels as K
from tune_conv import TILES, bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="fwd")
    for n, d in (("B", 256), ("H", 2), ("W", 2), ("cin", 256), ("cout", 256), ("k", 3), ("s", 1), ("p", 1)):
        ap.add_argument(f"--{n}", type=int, default=d)
    ap.add_argument("--stats", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda")
    B, H, W, ci, co, k, s, p = a.B, a.H, a.W, a.cin, a.cout, a.k, a.s, a.p
    OH, OW = K.out_hw(H, W, k, k, s, s, p, p)
    x = torch.randn(B, H, W, ci, device=dev).to(torch.bfloat16)
    w = (torch.randn(co, k, k, ci, device=dev) * 0.05).to(torch.bfloat16)
    dy = torch.randn(B, OH, OW, co, device=dev).to(torch.bfloat16)
    dw = torch.zeros(co, k, k, ci, device=dev)
    st = torch.zeros(2 * co, device=dev) if a.stats else None

    def run(cfg):
        if a.mode == "fwd":
            return K.conv_fwd(x, w, k, k, (s, s), (p, p), stats=st, cfg=cfg)
        if a.mode == "dgrad":
            return K.conv_dgrad(dy, w, x.shape, k, k, (s, s), (p, p), cfg=cfg)
        return K.conv_wgrad(x, dy, dw, k, k, (s, s), (p, p), cfg=cfg)
    res = []
    if a.mode != "wgrad":
        for bm, bn in ((16, 16), (16, 32), (32, 16), (32, 32), (32, 64), (64, 32), (64, 64)):
            for nw in (4, 8):
                cfg = (bm, bn, nw, 1, 3)
                try:
                    res.append((bench(lambda: run(cfg), reps=10), cfg))
                except Exception:
                    pass
    for bm, bn in TILES:
        for bk, var in ((32, 0), (64, 0), (64, 1), (64, 2)):
            for sp in (1, 2, 4, 8, 16, 32):
                cfg = (bm, bn, bk, sp, var)
                try:
                    t = bench(lambda: run(cfg), reps=10)
                except Exception as e:  # invalid combination
                    continue
                res.append((t, cfg))
    res.sort()
    top = int(os.environ.get("SWEEP_TOP", "25"))
    for t, cfg in res[:top]:
        print(f"{t:8.2f} us  {cfg}")
    print("worst", res[-1])


if __name__ == "__main__":
    main()
