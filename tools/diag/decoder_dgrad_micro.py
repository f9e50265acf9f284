"""The MLM decoder's input gradient (dx[2432, 768] = dy[2432, 30528] @ W[30528, 768], the one
BERT GEMM with few output tiles and a very long reduction) under several tiles / split-K counts
of the fp32-atomic split-K form, graph-free interleaved timing, median of rounds.

    python tools/diag/decoder_dgrad_micro.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    from kubeml_amd.ops import gemm as G
    from kubeml_amd.ops import kernels as K
    dev = torch.device("cuda", 0)
    T, ip, op = 2432, 768, 30528
    dy = torch.randn(T, op, device=dev).to(torch.bfloat16)
    w = (torch.randn(op, ip, device=dev) * 0.02).to(torch.bfloat16)
    acc = torch.empty(T, ip, dtype=torch.float32, device=dev)
    ref = (dy.float() @ w.float())
    cands = []
    for tile in ((128, 128, 2), (128, 128), (256, 128), (128, 256), (256, 256, 8), (256, 192, 8)):
        for s in (2, 4, 6, 8, 12, 16):
            cands.append((tile, s))
    ok = []
    for tile, s in cands:
        try:
            K.memset_(acc)
            G.gemm(dy, op, w, ip, acc, ip, T, ip, op, 1, 2, tile=tile, splits=s)
            torch.cuda.synchronize()
            err = float((acc - ref).abs().max() / ref.abs().max())
            if err < 1e-2:
                ok.append((tile, s))
            else:
                print(json.dumps({"tile": tile, "splits": s, "bad_rel": err}), flush=True)
        except Exception as e:   # tile without the split-K output form
            print(json.dumps({"tile": tile, "splits": s, "error": str(e)[:80]}), flush=True)
    times = {c: [] for c in ok}
    for _ in range(5):
        for tile, s in ok:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                K.memset_(acc)
                G.gemm(dy, op, w, ip, acc, ip, T, ip, op, 1, 2, tile=tile, splits=s)
            torch.cuda.synchronize()
            times[(tile, s)].append((time.perf_counter() - t0) / 10 * 1e6)
    for c in sorted(times, key=lambda c: sorted(times[c])[2]):
        print(json.dumps({"tile": "x".join(map(str, c[0])), "splits": c[1],
                          "us_incl_memset": round(sorted(times[c])[2], 1)}), flush=True)


if __name__ == "__main__":
    main()
