"""Run one kml_gemm configuration repeatedly (for rocprofv3 --pmc passes).

    python tools/gemm_one.py --layout 0 --M 16384 --N 3072 --K 768 --tile 256,256 --reps 20
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", type=int, default=0)
    ap.add_argument("--M", type=int, default=16384)
    ap.add_argument("--N", type=int, default=3072)
    ap.add_argument("--K", type=int, default=768)
    ap.add_argument("--tile", default="256,256")
    ap.add_argument("--splits", type=int, default=1)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--torch", action="store_true", help="run torch.mm (hipBLASLt) on the same operands instead")
    a = ap.parse_args()
    from kubeml_amd.ops import gemm as G
    dev = torch.device("cuda", 0)
    M, N, K = a.M, a.N, a.K
    tile = tuple(int(x) for x in a.tile.split(","))
    if a.layout == 0:
        A, B = torch.randn(M, K, device=dev).bfloat16(), torch.randn(N, K, device=dev).bfloat16()
        C, lda, ldb, out = torch.empty(M, N, dtype=torch.bfloat16, device=dev), K, K, 0
    elif a.layout == 1:
        A, B = torch.randn(M, K, device=dev).bfloat16(), torch.randn(K, N, device=dev).bfloat16()
        C, lda, ldb, out = torch.empty(M, N, dtype=torch.bfloat16, device=dev), K, N, 0
    else:
        A, B = torch.randn(K, M, device=dev).bfloat16(), torch.randn(K, N, device=dev).bfloat16()
        C, lda, ldb, out = torch.zeros(M, N, device=dev), M, N, (1 if a.splits == 1 else 2)
    for _ in range(a.reps):
        if a.torch:
            if a.layout == 0:
                torch.mm(A, B.t(), out=C)
            elif a.layout == 1:
                torch.mm(A, B, out=C)
            else:
                torch.addmm(C, A.t(), B, out_dtype=torch.float32)
            continue
        G.gemm(A, lda, B, ldb, C, N, M, N, K, a.layout, out, beta=1.0 if a.layout == 2 else 0.0, tile=tile,
               splits=a.splits)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
