"""1x1 stride-1 conv weight gradients at ResNet-50 shapes (batch 128): the implicit-GEMM conv
wgrad (current plan) vs gemm.hip's slab split-K GEMM vs hipBLASLt (torch.addmm, fp32 out,
beta 1).  Graph-timed; one JSON line per shape.

    python tools/wgrad_1x1.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch

from kubeml_amd.ops import gemm as G
from kubeml_amd.ops import kernels as K
from launch_floor import timed  # noqa: E402

SHAPES = [(401408, 64, 64), (401408, 64, 256), (401408, 256, 64), (401408, 128, 256),
          (100352, 128, 512), (100352, 512, 128), (100352, 256, 512),
          (25088, 256, 1024), (25088, 1024, 256), (25088, 512, 1024),
          (6272, 512, 2048), (6272, 2048, 512)]


def sweep():
    """--sweep: slab split-K tile x splits grid per shape; prints the best route per shape."""
    dev = torch.device("cuda")
    grid = {401408: [64, 96, 128, 192, 256, 384, 512], 100352: [32, 48, 64, 96, 128], 25088: [12, 16, 24, 32, 48],
            6272: [2, 3, 4, 6, 8, 12, 16]}
    if "--tiles" in sys.argv:    # the 128x128 two-stage tile only (it won every shape of the full sweep)
        tiles = [(128, 128, 2)]
    else:
        tiles = [(128, 128, 2), (256, 128), (128, 256), (256, 256, 8)]
    for P, Co, Ci in SHAPES:
        B = 128
        x2 = torch.randn(P, Ci, device=dev).to(torch.bfloat16)
        dy2 = torch.randn(P, Co, device=dev).to(torch.bfloat16)
        dw2 = torch.zeros(Co, Ci, device=dev)
        hw = int(round((P // B) ** 0.5))
        N = 4
        conv = timed(lambda: [K.conv_wgrad(x2.view(B, hw, hw, Ci), dy2.view(B, hw, hw, Co), dw2.view(Co, 1, 1, Ci),
                                           1, 1, (1, 1), (0, 0), cfg=K.plan_conv("wgrad", Co, Ci, P)) for _ in range(N)], N)
        best = ("conv", conv)
        res = {"P": P, "Cout": Co, "Cin": Ci, "conv_us": round(conv, 2)}
        for tile in tiles:
            for sp in grid[P]:
                t = timed(lambda: [G.wgrad_splitk_(dw2, dy2, Co, x2, Ci, Co, Ci, P, beta=0.0, tile=tile, splits=sp)
                                   for _ in range(N)], N)
                res[f"{'x'.join(map(str, tile))}/{sp}"] = round(t, 2)
                if t < best[1]:
                    best = (["slab", tile[0], tile[1], tile[2] if len(tile) > 2 else 0, sp], t)
        res["best"] = best[0]
        res["best_us"] = round(best[1], 2)
        print(json.dumps(res), flush=True)


def main():
    if "--sweep" in sys.argv:
        return sweep()
    dev = torch.device("cuda")
    for P, Co, Ci in SHAPES:
        torch.manual_seed(0)
        B = 128
        hw = int(round((P // B) ** 0.5))
        x = torch.randn(B, hw, hw, Ci, device=dev).to(torch.bfloat16)
        dy = torch.randn(B, hw, hw, Co, device=dev).to(torch.bfloat16)
        dw = torch.zeros(Co, 1, 1, Ci, device=dev)
        x2, dy2, dw2 = x.view(P, Ci), dy.view(P, Co), dw.view(Co, Ci)
        N = 4
        res = {"P": P, "Cout": Co, "Cin": Ci, "GF": round(2 * P * Co * Ci / 1e9, 2),
               "MB": round(2 * P * (Co + Ci) / 1e6, 1)}
        res["conv_us"] = round(timed(lambda: [K.conv_wgrad(x, dy, dw, 1, 1, (1, 1), (0, 0)) for _ in range(N)], N), 2)
        ref = dy2.double().t() @ x2.double()
        for tile in [(256, 256, 8), (128, 128, 2)]:
            for sp in [None, 32, 64, 128]:
                try:
                    t = timed(lambda: [G.wgrad_splitk_(dw2, dy2, Co, x2, Ci, Co, Ci, P, beta=0.0, tile=tile, splits=sp)
                                       for _ in range(N)], N)
                except Exception as e:  # noqa: BLE001
                    res[f"slab{tile[0]}_{sp}"] = str(e)[:60]
                    continue
                res[f"slab{tile[0]}_{sp}_us"] = round(t, 2)
        G.wgrad_splitk_(dw2, dy2, Co, x2, Ci, Co, Ci, P, beta=0.0, tile=(128, 128, 2))
        res["slab_rel"] = float((dw2.double() - ref).norm() / ref.norm())
        t = timed(lambda: [torch.addmm(dw2, dy2.t(), x2, out_dtype=torch.float32, out=dw2) for _ in range(N)], N)
        res["blas_us"] = round(t, 2)
        dw2.zero_()
        torch.addmm(dw2, dy2.t(), x2, out_dtype=torch.float32, out=dw2)
        res["blas_rel"] = float((dw2.double() - ref).norm() / ref.norm())
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
