"""Autotune the implicit-GEMM conv kernels for a model's exact layer shapes.

For every distinct (mode, M, N, Kd) of the model at the given batch, sweeps tile
(BM x BN), BK and split-K, times each config with hip events (median of N reps,
interleaved in one process as the CDNA guide's methodology asks), checks the
winner's output against the heuristic default config, and writes
``kubeml_amd/ops/conv_tuning.json`` which ``ops.kernels.plan_conv`` loads.

Usage (on the GPU box):  python tools/tune_conv.py --model resnet34 --batch 256
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from kubeml_amd.ops import kernels as K

TILES = [(32, 32), (32, 64), (64, 32), (64, 64), (64, 128), (128, 64), (128, 128), (32, 128), (128, 32),
         (256, 128), (128, 256)]  # the 256-wide tiles exist for the LDS-DMA variant only


def conv_layers(model_name, B, H=32, W=32, in_ch=3):
    from kubeml_amd import models
    from kubeml_amd.nn.modules import Conv2d, Linear
    m = models.get_model(model_name)
    shapes = []

    def hook(mod, inp, out):
        x = inp[0]
        if isinstance(mod, Conv2d):
            b, h, w, c = x.shape
            if K.unrolled22(h, w, mod.kernel_size[0], mod.kernel_size[1], mod.stride, mod.padding):
                # runs as its dense 1x1 form (ops.kernels.unrolled22): tune those GEMMs
                shapes.append(("conv", 4 * mod.cin_pad, 4 * mod.out_channels, 1, 1, 0, 1, 1))
                return
            shapes.append(("conv", mod.cin_pad, mod.out_channels, mod.kernel_size[0], mod.stride[0],
                           mod.padding[0], h, w))
        elif isinstance(mod, Linear):
            shapes.append(("linear", mod.in_pad, mod.out_pad, 1, 1, 0, 1, 1))

    hs = [mm.register_forward_hook(hook) for mm in m.modules() if isinstance(mm, (Conv2d, Linear))]
    m.eval()
    with torch.no_grad():
        m(torch.randn(2, in_ch, H, W))
    for h in hs:
        h.remove()
    uniq = []
    for s in shapes:
        if s not in uniq:
            uniq.append(s)
    return uniq


def bert_linears(B, L, P=76, hidden=768, inter=3072, vocab=30522):
    """(kind, cin, cout, k, s, p, H, W) entries for the BERT GEMMs as 1x1 convs over
    B*L tokens (and B*P masked positions for the MLM head)."""
    r8 = lambda c: -(-c // 8) * 8
    T, M = B * L, B * P
    out = []
    for (rows, fin, fout) in ((T, hidden, 3 * hidden), (T, hidden, hidden), (T, hidden, inter), (T, inter, hidden),
                              (M, hidden, hidden), (M, hidden, r8(vocab))):
        out.append(("linear", fin, fout, 1, 1, 0, 1, 1, rows))
    return out


def bench(fn, reps=20, warm=2, inner=10):
    """Device time per call: `inner` calls captured in a hipGraph (no host launch cost in
    the measurement — these kernels are shorter than a Python launch), replayed `reps`
    times; median over replays."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(inner):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record()
    for i in range(reps):
        g.replay()
        ev[i + 1].record()
    torch.cuda.synchronize()
    ts = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(reps))
    return ts[len(ts) // 2] * 1e3 / inner  # us per call


PAIR_DGRAD = [(32, 64, 64, sp, 0) for sp in (1, 2, 4)] + [(32, 32, 64, sp, 0) for sp in (1, 2, 4, 8)] + \
    [(32, 32, 4, 1, 3), (32, 16, 4, 1, 3), (64, 32, 4, 1, 3)]
PAIR_WGRAD = [(bm, 32, 64, sp, 0) for bm in (32, 64) for sp in (1, 2, 4, 8, 16, 32)]


def tune_pairs(layers, table, reps, dev):
    """Grouped dgrad+wgrad launches (ops.kernels.conv_bwd): for every conv layer time each
    instantiated (dgrad plan, wgrad plan) pair and keep the fastest when it beats the two
    separately tuned launches.  Entries: mode "pair", keyed by the dgrad and wgrad GEMMs."""
    out = []
    for (kind, cin, cout, k, s, p, H, W, B) in layers:
        if kind != "conv" or cin == 8:
            continue
        OH, OW = K.out_hw(H, W, k, k, s, s, p, p)
        r0, r1, s0, s1 = K.tap_window(H, W, k, k, s, s, p, p)
        ntap = (r1 - r0) * (s1 - s0)
        dkey = (B * H * W, cin, ntap * cout)
        wkey = (cout, ntap * cin, B * OH * OW)
        key = ("pair",) + dkey + wkey
        if key in table:
            continue
        x = torch.randn(B, H, W, cin, device=dev).to(torch.bfloat16)
        w = (torch.randn(cout, k, k, cin, device=dev) * 0.05).to(torch.bfloat16)
        dy = torch.randn(B, OH, OW, cout, device=dev).to(torch.bfloat16)
        dw = torch.zeros(cout, k, k, cin, device=dev)
        wt = torch.empty(cin, k, k, -(-cout // 32) * 32, dtype=torch.bfloat16, device=dev)
        K.weight_transpose_multi([w], [wt])
        sep_d = K.dgrad_plan(x.shape, cout, k, k, (s, s), (p, p))
        sep_w = K._norm_cfg(K.plan_conv("wgrad", *wkey))

        def sep():
            K.conv_wgrad(x, dy, dw, k, k, (s, s), (p, p), cfg=sep_w)
            K.conv_dgrad(dy, w, x.shape, k, k, (s, s), (p, p), cfg=sep_d)
        t_sep = bench(sep, reps=reps)
        res = []
        for dc in PAIR_DGRAD:
            if dc[4] == 0 and K.effective_splits(ntap * (-(-cout // 64) * 64), 64, dc[3]) != dc[3]:
                continue
            for wc in PAIR_WGRAD:
                if K.effective_splits(wkey[2], 64, wc[3]) != wc[3]:
                    continue
                if not K.conv_pair_supported(dc, wc):
                    continue
                try:
                    t = bench(lambda: K.conv_bwd(dy, w, x, dw, k, k, (s, s), (p, p), wt=wt, dcfg=dc, wcfg=wc),
                              reps=reps)
                except (RuntimeError, ValueError):
                    continue
                res.append((t, dc, wc))
        if not res:
            continue
        res.sort()
        t, dc, wc = res[0]
        # correctness of the winner vs the separate launches
        dw.zero_(); ref_x = K.conv_dgrad(dy, w, x.shape, k, k, (s, s), (p, p), cfg=sep_d).float()
        K.conv_wgrad(x, dy, dw, k, k, (s, s), (p, p), cfg=sep_w); ref_w = dw.clone()
        dw.zero_(); got_x = K.conv_bwd(dy, w, x, dw, k, k, (s, s), (p, p), wt=wt, dcfg=dc, wcfg=wc).float()
        err = max(((got_x - ref_x).norm() / (ref_x.norm() + 1e-12)).item(),
                  ((dw - ref_w).norm() / (ref_w.norm() + 1e-12)).item())
        entry = {"mode": "pair", "M": dkey[0], "N": dkey[1], "Kd": dkey[2], "wgrad": list(wkey),
                 "cfg": list(dc), "wcfg": list(wc), "us": round(t, 2), "separate_us": round(t_sep, 2),
                 "layer": [kind, cin, cout, k, s, p, H, W], "check_rel_err": err}
        if err < 1e-2:
            table[key] = entry
            out.append(entry)
        print(json.dumps(entry), flush=True)
    return out


def candidates(mode, M, N, Kd, cin, cout, ntap):
    """Every (bm, bn, bk, splits, variant) plan worth timing for one conv GEMM."""
    cands = []
    split_opts = [1, 2, 4, 8, 16] if mode != "wgrad" else [1, 2, 4, 8, 16, 32, 64]
    if mode != "wgrad" and M * N >= 256 * 256 * 64:
        split_opts = [1, 2]                 # thousands of output tiles: split-K only adds traffic
    elif mode == "wgrad" and Kd >= 32768:
        split_opts = [4, 8, 16, 32, 64]    # long reductions: never one block per tile
    for bm, bn in TILES:
        if bm > max(32, -(-M // 32) * 32) or bn > max(32, -(-N // 32) * 32):
            continue
        for bk, variant in ((32, 0), (64, 0), (64, 1), (64, 2)):
            for sp in split_opts:
                esp = K.effective_splits(Kd if mode != "dgrad" else ntap * (-(-cout // bk) * bk), bk, sp)
                if esp != sp:
                    continue
                cands.append((bm, bn, bk, sp, variant))
    if mode == "dgrad" or (mode == "fwd" and cin % 32 == 0):
        # LDS-free wave-split-K kernel (variant 3; the bk slot carries the wave count)
        for bm, bn in ((16, 16), (16, 32), (32, 16), (32, 32), (32, 64), (64, 32), (64, 64)):
            if bm > max(16, -(-M // 16) * 16) or bn > max(16, -(-N // 16) * 16):
                continue
            for nw in (4, 8):
                cands.append((bm, bn, nw, 1, 3))
    return cands


def save(args, table):
    out = {"model": "resnet34+bert_base" if args.bert else args.model, "batch": args.batch, "arch": "gfx950",
           "entries": sorted(table.values(), key=lambda e: (e["mode"], -e["M"]))}
    tmp = args.out + ".tmp"
    with open(tmp, "w") as f:
        json.dump(out, f, indent=1)
    os.replace(tmp, args.out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet34")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--out", default=K._TUNE_FILE)
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--bert", default=None, help="B,L: tune the BERT-base GEMM shapes instead of a CNN")
    ap.add_argument("--fresh", action="store_true", help="ignore existing entries (re-measure every shape)")
    ap.add_argument("--pairs", action="store_true", help="tune grouped dgrad+wgrad launches (conv layers)")
    ap.add_argument("--size", type=int, default=32, help="input image size of the CNN (224 for ImageNet shapes)")
    ap.add_argument("--max-seconds", type=float, default=0, help="stop (table saved) after this long")
    args = ap.parse_args()
    dev = torch.device("cuda")
    if args.bert:
        Bb, Lb = (int(v) for v in args.bert.split(","))
        layers = bert_linears(Bb, Lb)
    else:
        layers = [l + (args.batch,) for l in conv_layers(args.model, args.batch, H=args.size, W=args.size)]
    table = {}
    if os.path.exists(args.out) and not args.fresh:
        for e in json.load(open(args.out)).get("entries", []):
            if e["mode"] == "pair":
                table[("pair", e["M"], e["N"], e["Kd"]) + tuple(e["wgrad"])] = e
            else:
                table[(e["mode"], e["M"], e["N"], e["Kd"])] = e
    report = []
    t_start = time.time()
    if args.pairs:
        report = tune_pairs(layers, table, args.reps, dev)
        layers = []
    for (kind, cin, cout, k, s, p, H, W, B) in layers:
        OH, OW = K.out_hw(H, W, k, k, s, s, p, p)
        x = torch.randn(B, H, W, cin, device=dev).to(torch.bfloat16)
        w = (torch.randn(cout, k, k, cin, device=dev) * 0.05).to(torch.bfloat16)
        dy = torch.randn(B, OH, OW, cout, device=dev).to(torch.bfloat16)
        dw = torch.zeros(cout, k, k, cin, device=dev)
        stats = torch.zeros(2 * cout, device=dev)
        r0, r1, s0, s1 = K.tap_window(H, W, k, k, s, s, p, p)
        ntap = (r1 - r0) * (s1 - s0)
        shapes = {
            "fwd": (B * OH * OW, cout, ntap * cin),
            "dgrad": (B * H * W, cin, ntap * cout),
            "wgrad": (cout, ntap * cin, B * OH * OW),
        }
        for mode, (M, N, Kd) in shapes.items():
            if mode == "dgrad" and kind == "conv" and cin == 8:
                continue  # stem input never needs a gradient
            key = (mode, M, N, Kd)
            if key in table:
                continue

            def run(cfg, mode=mode):
                if mode == "fwd":
                    return K.conv_fwd(x, w, k, k, (s, s), (p, p), stats=stats, cfg=cfg)
                if mode == "dgrad":
                    return K.conv_dgrad(dy, w, x.shape, k, k, (s, s), (p, p), cfg=cfg)
                return K.conv_wgrad(x, dy, dw, k, k, (s, s), (p, p), cfg=cfg)

            default = K.default_plan(mode, M, N, Kd)
            cands = candidates(mode, M, N, Kd, cin, cout, ntap)
            res = []
            for cfg in cands:
                try:
                    res.append((bench(lambda: run(cfg), reps=args.reps), cfg))
                except (RuntimeError, ValueError):
                    pass
            res.sort()
            t_def = bench(lambda: run(default), reps=args.reps)
            best_t, best = res[0]
            # correctness of the winner vs the default config
            if mode == "wgrad":
                dw.zero_(); run(default); ref = dw.clone(); dw.zero_(); run(best); got = dw.clone()
            else:
                ref = run(default).float(); got = run(best).float()
            err = ((got - ref).norm() / (ref.norm() + 1e-12)).item()
            ok = err < 1e-2
            entry = {"mode": mode, "M": M, "N": N, "Kd": Kd, "cfg": list(best if ok else default),
                     "us": round(best_t if ok else t_def, 2), "default_us": round(t_def, 2),
                     "layer": [kind, cin, cout, k, s, p, H, W], "check_rel_err": err}
            table[key] = entry
            report.append(entry)
            print(json.dumps(entry), flush=True)
            save(args, table)                     # incremental: a cut-off run keeps its shapes
            if args.max_seconds and time.time() - t_start > args.max_seconds:
                break
        if args.max_seconds and time.time() - t_start > args.max_seconds:
            print(json.dumps({"stopped": "max-seconds"}), flush=True)
            break
    out = {"model": "resnet34+bert_base" if args.bert else args.model, "batch": args.batch, "arch": "gfx950",
           "entries": sorted(table.values(), key=lambda e: (e["mode"], -e["M"]))}
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    tot = sum(e["us"] for e in report)
    tdef = sum(e.get("default_us", e.get("separate_us", 0.0)) for e in report)
    print(json.dumps({"tuned_total_us": round(tot, 1), "default_total_us": round(tdef, 1),
                      "wall_s": round(time.time() - t_start, 1)}))


if __name__ == "__main__":
    main()
