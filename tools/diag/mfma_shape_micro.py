"""16x16x32 against 32x32x16 MFMA fragments on the same k_gemm tile (gemm.hip tiles 3 / 4 against
8 / 9: 128 x 128 block tile, 8 waves of 64 x 32, BK = 64, 3 or 2 LDS stages, register epilogue) on
BERT-base's forward (layout 0) GEMM shapes, bias + optional GELU as in the model.  Numerics are
checked against an fp32 torch matmul first; the timing is graph-free, interleaved, and the median
of rounds is reported.

    python tools/diag/mfma_shape_micro.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

SHAPES = [  # (name, M, N, K, act): 16384 tokens = BERT-base MLM bs 32 x 512
    ("qkv", 16384, 2304, 768, 0),
    ("attn_out", 16384, 768, 768, 0),
    ("ffn1_gelu", 16384, 3072, 768, 1),
    ("ffn2", 16384, 768, 3072, 0),
]
PAIRS = [((128, 128), (128, 128, 3, "mf32")), ((128, 128, 2), (128, 128, 2, "mf32"))]


def main():
    import torch
    from kubeml_amd.ops import gemm as G
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    rows = []
    for name, M, N, K, act in SHAPES:
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
        bias = torch.randn(N, device=dev) * 0.1
        ref = a.float() @ w.float().t() + bias
        if act:
            ref = torch.nn.functional.gelu(ref)
        c = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        tiles = [t for p in PAIRS for t in p]
        for t in tiles:
            c.zero_()
            G.gemm(a, K, w, K, c, N, M, N, K, 0, 0, bias=bias, act=act, tile=t, splits=1)
            torch.cuda.synchronize()
            err = float((c.float() - ref).abs().max() / ref.abs().max())
            if err > 1e-2:
                raise SystemExit(f"{name} tile {t}: rel err {err}")
        times = {t: [] for t in tiles}
        for _ in range(7):
            for t in tiles:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(20):
                    G.gemm(a, K, w, K, c, N, M, N, K, 0, 0, bias=bias, act=act, tile=t, splits=1)
                torch.cuda.synchronize()
                times[t].append((time.perf_counter() - t0) / 20 * 1e6)
        for m16, m32 in PAIRS:
            u16, u32 = sorted(times[m16])[3], sorted(times[m32])[3]
            r = {"shape": name, "M": M, "N": N, "K": K, "stages": 2 if len(m16) == 3 else 3,
                 "us_16x16x32": round(u16, 1), "us_32x32x16": round(u32, 1),
                 "tflops_16x16x32": round(2 * M * N * K / u16 / 1e6, 1),
                 "tflops_32x32x16": round(2 * M * N * K / u32 / 1e6, 1),
                 "ratio_32_over_16": round(u32 / u16, 3)}
            rows.append(r)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
