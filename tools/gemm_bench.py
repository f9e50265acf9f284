"""Hand-written MFMA GEMM vs hipBLASLt (torch.mm) on the BERT-base linear shapes.

For every (layout, M, N, K) of BERT-base at T = batch x seq tokens — forward (y = x W^T),
dgrad (dx = dy W) and wgrad (dW += dy^T x, fp32) of the QKV, attention-output, FFN1 and
FFN2 linears and the MLM transform — times every tile / split-K of kml_gemm and the
torch reference (interleaved rounds in one process, median of rounds; CDNA guide §5.4
rule 24), on random data.  Writes the winners to kubeml_amd/ops/gemm_tuning.json
(--write PATH) and prints one JSON line per shape.

    python tools/gemm_bench.py --tokens 16384 [--write gpurun_out/gemm_tuning.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def shapes(T, hidden=768, inter=3072):
    lin = {"qkv": (hidden, 3 * hidden), "attn_out": (hidden, hidden), "ffn1": (hidden, inter),
           "ffn2": (inter, hidden)}
    out = []
    for name, (ip, op) in lin.items():
        out.append((name, 0, T, op, ip))      # forward: M=T, N=op, K=ip
        out.append((name, 1, T, ip, op))      # dgrad: M=T, N=ip, K=op
        out.append((name, 2, op, ip, T))      # wgrad: M=op, N=ip, K=T
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--write", default=None, help="write the winners to this tuning json")
    ap.add_argument("--shapes", default=None, help="custom shapes 'layout:M:N:K;...' instead of BERT's")
    ap.add_argument("--tiles", default="all", help="comma list of tile names to try, e.g. 256x256x8,128x128x2")
    a = ap.parse_args()
    from kubeml_amd.ops import gemm as G
    dev = torch.device("cuda", 0)
    T = a.tokens
    entries, rows = [], []
    todo = shapes(T)
    if a.shapes:
        todo = [("custom", *[int(v) for v in sh.split(":")]) for sh in a.shapes.split(";")]
    for name, layout, M, N, K in todo:
        # operands in their natural buffers
        if layout == 0:
            A = torch.randn(M, K, device=dev).to(torch.bfloat16)              # x [T][ip]
            B = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)     # W [op][ip]
            C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            lda, ldb, out = K, K, 0
            ref = lambda: torch.mm(A, B.t())
        elif layout == 1:
            A = torch.randn(M, K, device=dev).to(torch.bfloat16)              # dy [T][op]
            B = (torch.randn(K, N, device=dev) * 0.05).to(torch.bfloat16)     # W [op][ip]
            C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            lda, ldb, out = K, N, 0
            ref = lambda: torch.mm(A, B)
        else:
            A = torch.randn(K, M, device=dev).to(torch.bfloat16)              # dy [T][op]
            B = torch.randn(K, N, device=dev).to(torch.bfloat16)              # x [T][ip]
            C = torch.zeros(M, N, dtype=torch.float32, device=dev)
            lda, ldb, out = M, N, 1
            ref = lambda: torch.addmm(C, A.t(), B, out_dtype=torch.float32)
        cands = []
        for tile in ((256, 256), (256, 256, 4), (256, 256, 8), (256, 192, 8), (256, 128), (128, 256), (128, 128),
                     (128, 128, 2), (128, 128, 3, "mf32"), (128, 128, 2, "mf32")):
            tname = "x".join(str(v) for v in tile)
            if a.tiles != "all" and tname not in a.tiles.split(","):
                continue
            if tile[-1] == "mf32" and layout != 0:   # the 32x32x16 form: forward layout only
                continue
            for s in ((1,) if layout != 2 else (1, 2, 4, 8, 16)):
                if layout == 2 and s > 1 and K // s < 256:
                    continue
                cands.append((tile, s))
            if layout == 2:   # deterministic slab split-K (kml_gemm_wgrad_splitk)
                tiles = -(-M // tile[0]) * -(-N // tile[1])
                base = max(1, round(256 / tiles))
                for s in sorted({max(1, base // 2), base, base * 2, base * 4, base * 8}):
                    if K // s >= 256:
                        cands.append((tile + ("slab",), s))

        def run(tile, s):
            if tile[-1] == "slab":
                G.wgrad_splitk_(C, A, lda, B, ldb, M, N, K, beta=1.0, tile=tile[:-1], splits=s)
                return
            G.gemm(A, lda, B, ldb, C, N, M, N, K, layout, out if s == 1 else 2, beta=1.0 if layout == 2 else 0.0,
                   tile=tile, splits=s)
        nm = lambda t, s: (f"{t[0]}x{t[1]}" + (f"x{t[2]}st" if len(t) > 2 and t[2] != "slab" else "")
                           + ("-mf32" if t[-1] == "mf32" else "")
                           + (f"/k{s}" if t[-1] == "slab" else f"/s{s}"))
        fns = [("torch", ref)] + [(nm(t, s), (lambda t=t, s=s: run(t, s))) for t, s in cands]
        for _, f in fns:
            f()
        torch.cuda.synchronize()
        times = {n: [] for n, _ in fns}
        for _ in range(a.rounds):
            for n, f in fns:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.reps):
                    f()
                torch.cuda.synchronize()
                times[n].append((time.perf_counter() - t0) / a.reps * 1e6)
        med = {n: sorted(v)[len(v) // 2] for n, v in times.items()}
        best = min((n for n in med if n != "torch"), key=lambda n: med[n])
        flop = 2.0 * M * N * K
        t_best, s_best = cands[[nm(t, s) for t, s in cands].index(best)]
        row = {"shape": name, "layout": ["fwd", "dgrad", "wgrad"][layout], "M": M, "N": N, "K": K,
               "torch_us": round(med["torch"], 1), "torch_TF": round(flop / med["torch"] / 1e6, 1),
               "best": best, "best_us": round(med[best], 1), "best_TF": round(flop / med[best] / 1e6, 1),
               "speedup_vs_torch": round(med["torch"] / med[best], 3),
               "all_us": {n: round(v, 1) for n, v in med.items()}}
        rows.append(row)
        print(json.dumps(row), flush=True)
        entries.append({"layout": layout, "M": M, "N": N, "K": K, "tile": list(t_best), "splits": s_best,
                        "us": round(med[best], 1), "torch_us": round(med["torch"], 1)})
    tot_t = sum(r["torch_us"] for r in rows)
    tot_b = sum(r["best_us"] for r in rows)
    print(json.dumps({"summary": True, "tokens": T, "sum_torch_us": round(tot_t, 1), "sum_kml_us": round(tot_b, 1),
                      "speedup": round(tot_t / tot_b, 3)}), flush=True)
    if a.write:
        path = a.write
        old = []
        if os.path.exists(path):
            with open(path) as f:
                old = [e for e in json.load(f).get("entries", [])
                       if (e["layout"], e["M"], e["N"], e["K"]) not in {(x["layout"], x["M"], x["N"], x["K"])
                                                                         for x in entries}]
        with open(path, "w") as f:
            json.dump({"entries": old + entries}, f, indent=1)


if __name__ == "__main__":
    main()
