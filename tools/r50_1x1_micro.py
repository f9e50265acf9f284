"""Graph-timed ResNet-50 1x1 forward convs (batch 128, 224^2 shapes) against the bytes they move.

For each 1x1 conv: our conv_fwd with the BN partial-statistics epilogue (as the model runs it),
without statistics, every tuned tile of the implicit GEMM, hipBLASLt (torch.mm of the same GEMM)
and a write-only fill of the output (the HBM floor of the store side).

Usage (GPU box):  python tools/r50_1x1_micro.py [--tiles]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from kubeml_amd.ops import kernels as K
from tools.conv_micro import gtime

SHAPES = [  # B, H, Cin, Cout, stride (every 1x1 forward conv of ResNet-50 at 224^2)
    (128, 56, 64, 256, 1),
    (128, 56, 64, 64, 1),
    (128, 56, 256, 64, 1),
    (128, 56, 256, 128, 1),
    (128, 56, 256, 512, 2),
    (128, 28, 128, 512, 1),
    (128, 28, 512, 128, 1),
    (128, 28, 512, 256, 1),
    (128, 28, 512, 1024, 2),
    (128, 14, 256, 1024, 1),
    (128, 14, 1024, 256, 1),
    (128, 14, 1024, 512, 1),
    (128, 14, 1024, 2048, 2),
    (128, 7, 512, 2048, 1),
    (128, 7, 2048, 512, 1),
]
TILES = [(32, 64), (64, 32), (64, 64), (128, 32), (128, 64), (64, 128), (128, 128), (256, 128), (128, 256)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", action="store_true", help="also time every implicit-GEMM tile")
    ap.add_argument("--gemm", action="store_true", help="also time the plain MFMA GEMM (ops.gemm) tiles, no stats")
    ap.add_argument("--route", action="store_true", help="time the conv GEMM route (BN stats epilogue) per tile")
    ap.add_argument("--conv3", action="store_true", help="3x3 forward convs: implicit GEMM vs the GEMM gather route")
    ap.add_argument("--wgrad3", action="store_true", help="3x3 weight gradients: implicit GEMM vs the gather route")
    ap.add_argument("--stem", action="store_true", help="with --wgrad3: the 7x7/s2 stem's weight gradient instead")
    ap.add_argument("--vgg", action="store_true", help="with --conv3 / --wgrad3: VGG-16 (CIFAR) 3x3 shapes")
    ap.add_argument("--dgrad", action="store_true", help="time the 1x1 dgrads (consumer-BN epilogue, residual addend "
                                                          "where the model has one) against the plain GEMM")
    args = ap.parse_args()
    dev = torch.device("cuda")
    if args.dgrad:
        return dgrad_main(dev)
    if args.conv3:
        return conv3_main(dev, args.vgg)
    if args.wgrad3:
        return wgrad3_main(dev, args.stem, args.vgg)
    for (B, H, C, Co, st) in SHAPES:
        x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(Co, 1, 1, C, device=dev) * 0.05).to(torch.bfloat16)
        OH = (H - 1) // st + 1
        y = torch.empty(B, OH, OH, Co, dtype=torch.bfloat16, device=dev)
        M = B * OH * OH
        S = (st, st)
        plan = K.conv_fwd_plan(C, M, Co, C, geom=(H, H, 1, 1, S, (0, 0)))
        G = K.conv_fwd_stats_rows(x.shape, Co, 1, 1, S, (0, 0))
        rows = torch.empty(G * 2 * Co, device=dev)
        t_st = gtime(lambda: K.conv_fwd(x, w, 1, 1, S, (0, 0), out=y, stats=rows, stats_part=True))
        t_ns = gtime(lambda: K.conv_fwd(x, w, 1, 1, S, (0, 0), out=y))
        A = x[:, ::st, ::st, :].contiguous().view(M, C)
        Bm = w.view(Co, C).t()
        C_ = y.view(M, Co)
        t_mm = gtime(lambda: torch.mm(A, Bm, out=C_))
        t_fill = gtime(lambda: y.fill_(1.0))
        byts = (x.numel() + y.numel()) * 2
        fl = 2 * M * Co * C
        best = (t_st, plan)
        print(f"1x1 {H}x{H}/s{st} {C}->{Co} M={M} plan={plan} G={G}: ours+stats {t_st:.1f}us "
              f"({byts / t_st / 1e6:.2f} TB/s, {fl / t_st / 1e6:.0f} TF/s)  ours {t_ns:.1f}us  "
              f"hipblaslt {t_mm:.1f}us  fill(out) {t_fill:.1f}us  [bytes {byts / 1e6:.0f} MB]", flush=True)
        if args.gemm and st == 1:
            from kubeml_amd.ops import gemm as G
            for tile in G.TILES:
                if tile[0] > M or tile[1] > Co:
                    continue
                try:
                    t = gtime(lambda: G.gemm(A, C, w.view(Co, C), C, C_, Co, M, Co, C, 0, 0, tile=tile, splits=1),
                              reps=20)
                except Exception as e:
                    print(f"   gemm {tile}: n/a ({str(e)[:60]})", flush=True)
                    continue
                print(f"   gemm {tile}: {t:.1f}us ({byts / t / 1e6:.2f} TB/s, {fl / t / 1e6:.0f} TF/s)", flush=True)
        if args.route and st == 1:
            rbest = None
            for (bm, bn, tc) in sorted(K._GEMM1X1_TILES):
                cfg = (bm, bn, tc, 1, K.GEMM1X1)
                G2 = K.conv_fwd_stats_rows(x.shape, Co, 1, 1, S, (0, 0), cfg=cfg)
                r2 = torch.empty(G2 * 2 * Co, device=dev)
                t = gtime(lambda: K.conv_fwd(x, w, 1, 1, S, (0, 0), out=y, stats=r2, stats_part=True, cfg=cfg),
                          reps=20)
                print(f"   route {cfg}: {t:.1f}us ({byts / t / 1e6:.2f} TB/s, {fl / t / 1e6:.0f} TF/s)", flush=True)
                if rbest is None or t < rbest[0]:
                    rbest = (t, cfg)
            print(f"ROUTE fwd M={M} N={Co} Kd={C}: {rbest[1]} {rbest[0]:.1f}us (plan {plan} {t_st:.1f}us)",
                  flush=True)
        if args.tiles:
            for (bm, bn) in TILES:
                for bk, var in [(32, 0), (64, 0), (64, 1)]:
                    if bk > C or bn > Co or ((bm == 256 or bn == 256) and var != 1):
                        continue
                    cfg = (bm, bn, bk, 1, var)
                    try:
                        G2 = K.conv_fwd_stats_rows(x.shape, Co, 1, 1, S, (0, 0), cfg=cfg)
                        r2 = torch.empty(G2 * 2 * Co, device=dev)
                        t = gtime(lambda: K.conv_fwd(x, w, 1, 1, S, (0, 0), out=y, stats=r2,
                                                     stats_part=True, cfg=cfg), reps=20)
                    except Exception as e:  # tile not instantiated for this variant
                        print(f"   cfg {cfg}: n/a ({str(e)[:60]})", flush=True)
                        continue
                    print(f"   cfg {cfg}: {t:.1f}us ({byts / t / 1e6:.2f} TB/s)", flush=True)
                    if t < best[0]:
                        best = (t, cfg)
            print(f"BEST fwd M={M} N={Co} Kd={C}: {best[1]} {best[0]:.1f}us (plan {t_st:.1f}us)", flush=True)


CONV3 = [  # B, H, C, K, stride: the 3x3 convs of ResNet-50 at 224^2
    (128, 56, 64, 64, 1), (128, 56, 128, 128, 2), (128, 28, 128, 128, 1), (128, 28, 256, 256, 2),
    (128, 14, 256, 256, 1), (128, 14, 512, 512, 2), (128, 7, 512, 512, 1)]


VGG3 = [  # B, H, C, K, stride: VGG-16 (CIFAR, batch 128) 3x3 convs with C % 64 == 0
    (128, 32, 64, 64, 1), (128, 16, 64, 128, 1), (128, 16, 128, 128, 1), (128, 8, 128, 256, 1),
    (128, 8, 256, 256, 1), (128, 4, 256, 512, 1), (128, 4, 512, 512, 1)]


def conv3_main(dev, vgg=False):
    for (B, H, C, Co, st) in (VGG3 if vgg else CONV3):
        x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(Co, 3, 3, C, device=dev) * 0.02).to(torch.bfloat16)
        S, P = (st, st), (1, 1)
        OH = (H - 1) // st + 1
        M = B * OH * OH
        y = torch.empty(B, OH, OH, Co, dtype=torch.bfloat16, device=dev)
        plan = K.conv_fwd_plan(C, M, Co, 9 * C, geom=(H, H, 3, 3, S, P))
        G = K.conv_fwd_stats_rows(x.shape, Co, 3, 3, S, P)
        rows = torch.empty(G * 2 * Co, device=dev)
        t = gtime(lambda: K.conv_fwd(x, w, 3, 3, S, P, out=y, stats=rows, stats_part=True), reps=20)
        fl = 2 * M * Co * 9 * C
        line = f"conv3 {H}x{H}/s{st} {C}->{Co} M={M} plan={plan}: {t:.1f}us ({fl / t / 1e6:.0f} TF/s)"
        best = None
        for (bm, bn, tc) in sorted(K._GEMM1X1_TILES):
            if tc > 4:
                continue
            cfg = (bm, bn, tc, 1, K.GEMM1X1)
            G2 = K.conv_fwd_stats_rows(x.shape, Co, 3, 3, S, P, cfg=cfg)
            r2 = torch.empty(G2 * 2 * Co, device=dev)
            tg = gtime(lambda: K.conv_fwd(x, w, 3, 3, S, P, out=y, stats=r2, stats_part=True, cfg=cfg), reps=20)
            line += f"  g{cfg[:3]}: {tg:.1f}"
            if best is None or tg < best[0]:
                best = (tg, cfg)
        print(line, flush=True)
        print(f"C3ROUTE fwd M={M} N={Co} Kd={9 * C}: {best[1]} {best[0]:.1f}us (plan {plan} {t:.1f}us) "
              f"[{fl / best[0] / 1e6:.0f} TF/s]", flush=True)
        if st != 1:
            continue
        # input gradient with the consumer-BN epilogue (as the model runs it)
        dy = torch.randn(B, H, H, Co, device=dev).to(torch.bfloat16)
        xs = (B, H, H, C)
        yb = torch.randn(xs, device=dev).to(torch.bfloat16)
        cb = torch.randn(xs, device=dev).to(torch.bfloat16)
        mean, rstd = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        out = torch.empty(xs, dtype=torch.bfloat16, device=dev)
        dplan = K.plan_conv("dgrad", B * H * H, C, 9 * Co)
        td = gtime(lambda: K.conv_dgrad(dy, w, xs, 3, 3, S, P, out=out, bnf=(yb, cb, mean, rstd), bnf_mask=True),
                   reps=20)
        dbest = None
        line = f"dgrad3 {H}x{H} {Co}->{C} plan={dplan}: {td:.1f}us"
        for (bm, bn, tc) in sorted(K._GEMM1X1_TILES):
            if tc > 4:
                continue
            cfg = (bm, bn, tc, 1, K.GEMM1X1)
            tg = gtime(lambda: K.conv_dgrad(dy, w, xs, 3, 3, S, P, out=out, cfg=cfg, bnf=(yb, cb, mean, rstd),
                                            bnf_mask=True), reps=20)
            line += f"  g{cfg[:3]}: {tg:.1f}"
            if dbest is None or tg < dbest[0]:
                dbest = (tg, cfg)
        print(line, flush=True)
        print(f"D3ROUTE dgrad M={B * H * H} N={C} Kd={9 * Co}: {dbest[1]} {dbest[0]:.1f}us (plan {dplan} {td:.1f}us) "
              f"[{fl / dbest[0] / 1e6:.0f} TF/s]", flush=True)


def wgrad3_main(dev, stem=False, vgg=False):
    shapes = [(128, 224, 8, 64, 2, 7)] if stem else [c + (3,) for c in (VGG3 if vgg else CONV3)]
    for (B, H, C, Co, st, kk) in shapes:
        x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
        pd = (kk - 1) // 2
        OH = (H + 2 * pd - kk) // st + 1
        dy = torch.randn(B, OH, OH, Co, device=dev).to(torch.bfloat16)
        dw = torch.zeros(Co, kk, kk, C, device=dev)
        S, P = (st, st), (pd, pd)
        t = gtime(lambda: K.conv_wgrad(x, dy, dw, kk, kk, S, P, accumulate=True), reps=10)
        fl = 2 * B * OH * OH * Co * kk * kk * C
        line = f"wgrad3 {H}x{H}/s{st} {C}->{Co}: {t:.1f}us ({fl / t / 1e6:.0f} TF/s)"
        best = None
        key = (B * H * H, Co, C, kk, st)
        for (bm, bn, stg) in [(128, 128, 2), (128, 128, 0), (256, 128, 0), (128, 256, 0)]:
            for sp in ((128, 256, 512) if stem else (8, 16, 32, 64, 128)):
                route = ("gather", bm, bn, stg, sp)
                K._WGRAD_GEMM[key] = route
                tg = gtime(lambda: K.conv_wgrad(x, dy, dw, kk, kk, S, P, accumulate=True), reps=10)
                del K._WGRAD_GEMM[key]
                line += f" {bm}x{bn}s{stg}/{sp}:{tg:.1f}"
                if best is None or tg < best[0]:
                    best = (tg, route)
        print(line, flush=True)
        print(f"W3ROUTE P={B * H * H} K={Co} C={C} KH={kk} S={st}: {list(best[1])} {best[0]:.1f}us (implicit {t:.1f}us) "
              f"[{fl / best[0] / 1e6:.0f} TF/s]", flush=True)


def dgrad_main(dev):
    from kubeml_amd.ops import gemm as G
    for (B, H, C, Co, st) in SHAPES:
        if st != 1:
            continue
        for addend in (False, True, None):   # None: plain dgrad (no consumer BN, no addend)
            dy = torch.randn(B, H, H, Co, device=dev).to(torch.bfloat16)
            w = (torch.randn(Co, 1, 1, C, device=dev) * 0.05).to(torch.bfloat16)
            xs = (B, H, H, C)
            yb = torch.randn(xs, device=dev).to(torch.bfloat16)
            cb = torch.randn(xs, device=dev).to(torch.bfloat16)
            mean = torch.zeros(C, device=dev)
            rstd = torch.ones(C, device=dev)
            add = torch.randn(xs, device=dev).to(torch.bfloat16) if addend else None
            bnfa = None if addend is None else (yb, cb, mean, rstd)
            out = torch.empty(xs, dtype=torch.bfloat16, device=dev)
            M = B * H * H
            plan = K.plan_conv("dgrad", M, C, Co)
            t = gtime(lambda: K.conv_dgrad(dy, w, xs, 1, 1, (1, 1), (0, 0), out=out, addend=add,
                                           bnf=bnfa, bnf_mask=True), reps=20)
            byts = (dy.numel() + 3 * out.numel() + (out.numel() if addend else 0)) * 2
            fl = 2 * M * Co * C
            line = (f"dgrad 1x1 {H}x{H} {Co}->{C} M={M} addend={addend} plan={plan}: {t:.1f}us "
                    f"({byts / t / 1e6:.2f} TB/s, {fl / t / 1e6:.0f} TF/s)")
            best = None
            for (bm, bn, tc) in sorted(K._GEMM1X1_TILES):
                if tc > 4:
                    continue
                cfg = (bm, bn, tc, 1, K.GEMM1X1)
                tg = gtime(lambda: K.conv_dgrad(dy, w, xs, 1, 1, (1, 1), (0, 0), out=out, addend=add, cfg=cfg,
                                                bnf=bnfa, bnf_mask=True), reps=20)
                line += f"  route{cfg[:3]}: {tg:.1f}"
                if best is None or tg < best[0]:
                    best = (tg, cfg)
            print(line, flush=True)
            print(f"DROUTE dgrad M={M} N={C} Kd={Co} addend={addend}: {best[1]} {best[0]:.1f}us (plan {plan} {t:.1f}us)",
                  flush=True)


if __name__ == "__main__":
    main()
