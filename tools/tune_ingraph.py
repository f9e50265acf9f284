"""In-graph conv plan tuning for the headline ResNet-34 step.

``tools/tune_conv.py`` times every plan of a conv GEMM in isolation (the same kernel replayed
back to back, its operands hot in L2).  Inside the training step the ranking changes: each
kernel's inputs were just written by another kernel (often on another XCD, so they come from
the Infinity Cache or HBM), the fp32 weight-gradient atomics land on lines the step's
zero-fill evicted, and a plan that needs a transposed weight copy pays for it at the start of
the step.  Measured on MI355X: an isolated-best pair table made the step 6 % SLOWER than the
table it replaced.  So this tool ranks plans by what they do to the whole step:

1. For each distinct conv GEMM of the model (fwd / dgrad / wgrad; unrolled 2x2-map convs in
   their 1x1 form) rank the plans in isolation (tune_conv.bench) and keep the top ``--topk``
   plus the plan the current table runs.
2. Build and capture the headline step (bench.py's config: batch 256, SGD, on-device
   augmentation, one hipGraph), time ``--steps`` replays with HIP events.
3. Coordinate descent: per forward GEMM, then per conv's backward (dgrad x wgrad plan pair,
   grouped into one launch when an instantiated pair exists), install each candidate,
   re-capture, time; keep it when the step gets faster by more than ``--min-gain``.
4. Write the table in tune_conv's format (``--out``).

Usage (GPU box):  python tools/tune_ingraph.py --out gpurun_out/conv_tuning.json
"""
import argparse
import gc
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch

from kubeml_amd.ops import kernels as K
import tune_conv as TC

CIFAR_TRAIN = 50000


def build_step(B, dev, lr=0.01):
    from kubeml_amd.engine.dp import make_train_step
    from kubeml_amd.models.resnet import resnet34
    from kubeml_amd.nn import cross_entropy, flatten_module
    from kubeml_amd.optim import SGD
    g = torch.Generator(device=dev).manual_seed(0)
    data = torch.randint(0, 256, (CIFAR_TRAIN, 32, 32, 3), dtype=torch.uint8, device=dev, generator=g)
    labels = torch.randint(0, 10, (CIFAR_TRAIN,), dtype=torch.int64, device=dev, generator=g)
    ctr = torch.tensor([1000.0, 0.0, 0.0], dtype=torch.float32, device=dev)
    xbuf = torch.empty((B, 32, 32, 8), dtype=torch.bfloat16, device=dev)
    ybuf = torch.empty((B,), dtype=torch.int64, device=dev)
    torch.manual_seed(0)
    model = resnet34(num_classes=1000).to(dev)
    space = flatten_module(model)
    model.train()
    opt = SGD(model.parameters(), lr=lr, weight_decay=1e-4)

    def make():
        return make_train_step(
            model, space, opt, cross_entropy, xbuf, ybuf,
            pre=lambda: K.augment(data, labels, ctr, B, out=xbuf, labels_out=ybuf, train=True),
            post=lambda: K.advance_counter_(ctr, B, CIFAR_TRAIN), world=1, use_graph=True, extra_state=[ctr])
    return model, make


class StepTimer:
    """Captures the step with the current plan tables; times captured steps.  Plans are baked
    into a graph at capture, so an incumbent and a candidate graph can be replayed
    alternately (A/B/A/B...) without re-capturing: clock drift cancels out."""

    def __init__(self, model, make, steps, warmup=10):
        self.model, self.make, self.steps, self.warmup = model, make, steps, warmup

    def _reset_flags(self):
        from kubeml_amd.nn.modules import Conv2d
        for m in self.model.modules():
            if isinstance(m, Conv2d):
                object.__setattr__(m, "_kml_wants_wt", False)
                object.__setattr__(m, "_kml_wt", None)

    def capture(self):
        gc.collect()
        torch.cuda.synchronize()
        self._reset_flags()
        # one eager step marks the convs that need derived weights, then the real capture
        st = self.make()
        st()
        torch.cuda.synchronize()
        st = self.make()
        st.capture()
        for _ in range(self.warmup):
            st()
        return st

    def time(self, st):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(self.steps):
            st()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / self.steps

    def ab(self, a, b, rounds):
        ta, tb = [], []
        for _ in range(rounds):
            ta.append(self.time(a))
            tb.append(self.time(b))
        ta.sort()
        tb.sort()
        return ta[len(ta) // 2], tb[len(tb) // 2]


def rank_isolated(layer, mode, B, dev, topk, reps):
    kind, cin, cout, k, s, p, H, W = layer
    OH, OW = K.out_hw(H, W, k, k, s, s, p, p)
    r0, r1, s0, s1 = K.tap_window(H, W, k, k, s, s, p, p)
    ntap = (r1 - r0) * (s1 - s0)
    M, N, Kd = {"fwd": (B * OH * OW, cout, ntap * cin), "dgrad": (B * H * W, cin, ntap * cout),
                "wgrad": (cout, ntap * cin, B * OH * OW)}[mode]
    x = torch.randn(B, H, W, cin, device=dev).to(torch.bfloat16)
    w = (torch.randn(cout, k, k, cin, device=dev) * 0.05).to(torch.bfloat16)
    dy = torch.randn(B, OH, OW, cout, device=dev).to(torch.bfloat16)
    dw = torch.zeros(cout, k, k, cin, device=dev)
    stats = torch.zeros(2 * cout, device=dev)

    def run(cfg):
        if mode == "fwd":
            return K.conv_fwd(x, w, k, k, (s, s), (p, p), stats=stats, cfg=cfg)
        if mode == "dgrad":
            return K.conv_dgrad(dy, w, x.shape, k, k, (s, s), (p, p), cfg=cfg)
        return K.conv_wgrad(x, dy, dw, k, k, (s, s), (p, p), cfg=cfg)
    res = []
    for cfg in TC.candidates(mode, M, N, Kd, cin, cout, ntap):
        try:
            res.append((TC.bench(lambda: run(cfg), reps=reps), tuple(cfg)))
        except (RuntimeError, ValueError):
            pass
    res.sort()
    return (M, N, Kd), [c for _, c in res[:topk]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--topk", type=int, default=3)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--min-gain", type=float, default=0.003, help="relative step-time gain to accept a plan")
    ap.add_argument("--rounds", type=int, default=4, help="A/B rounds per candidate")
    ap.add_argument("--out", default="gpurun_out/conv_tuning.json")
    ap.add_argument("--only", default="fwd,bwd", help="which passes to tune")
    args = ap.parse_args()
    dev = torch.device("cuda")
    t_start = time.time()
    B = args.batch
    layers = TC.conv_layers("resnet34", B)
    model, make = build_step(B, dev)
    timer = StepTimer(model, make, args.steps)
    inc = timer.capture()
    base = timer.time(inc)
    print(json.dumps({"start_ms": round(base, 4), "layers": len(layers)}), flush=True)

    def plan_of(mode, key):
        return tuple(K._norm_cfg(K.plan_conv(mode, *key)))

    def accept(label, cands, install, current):
        """A/B every candidate against the incumbent graph; keep the winner installed."""
        nonlocal inc, base
        best = current
        for c in cands:
            if c == current or c == best:
                continue
            install(c)
            try:
                cand = timer.capture()
            except (RuntimeError, ValueError) as e:
                print(json.dumps({"shape": label, "cand": c, "error": str(e)[:120]}), flush=True)
                install(best)
                continue
            ti, tc = timer.ab(inc, cand, args.rounds)
            print(json.dumps({"shape": label, "cand": c, "ms": round(tc, 4), "incumbent_ms": round(ti, 4)}),
                  flush=True)
            if tc < ti * (1 - args.min_gain):
                best, inc, base = c, cand, tc
            else:
                del cand
            install(best)
        print(json.dumps({"shape": label, "chosen": best, "ms": round(base, 4)}), flush=True)
        return best

    if "fwd" in args.only:
        for layer in layers:
            key, cands = rank_isolated(layer, "fwd", B, dev, args.topk, args.reps)
            cur = plan_of("fwd", key)

            def install(c, key=key):
                K._TUNED[("fwd",) + key] = tuple(c)
            accept(f"fwd{key}", cands, install, cur)

    if "bwd" in args.only:
        for layer in layers:
            if layer[0] != "conv":
                continue
            if layer[1] == 8:   # stem: no input gradient, the weight gradient runs alone
                wkey, wc = rank_isolated(layer, "wgrad", B, dev, args.topk, args.reps)

                def install_w(c, wkey=wkey):
                    K._TUNED[("wgrad",) + wkey] = tuple(c)
                accept(f"wgrad{wkey}", wc, install_w, plan_of("wgrad", wkey))
                continue
            dkey, dc = rank_isolated(layer, "dgrad", B, dev, args.topk, args.reps)
            wkey, wc = rank_isolated(layer, "wgrad", B, dev, args.topk, args.reps)
            pkey = dkey + wkey
            cur = K._TUNED_PAIR.get(pkey) or (plan_of("dgrad", dkey), plan_of("wgrad", wkey))
            cur = (tuple(cur[0]), tuple(cur[1]))
            combos = [(d, w) for d in dc for w in wc]

            def install(c, pkey=pkey):
                K._TUNED_PAIR[pkey] = (tuple(c[0]), tuple(c[1]))
            accept(f"bwd{pkey}", combos, install, cur)

    # write the table: current singles + pairs
    old = {}
    if os.path.exists(K._TUNE_FILE):
        old = json.load(open(K._TUNE_FILE))
    ents = {}
    for e in old.get("entries", []):
        key = ("pair", e["M"], e["N"], e["Kd"]) + tuple(e["wgrad"]) if e["mode"] == "pair" else \
            (e["mode"], e["M"], e["N"], e["Kd"])
        ents[key] = e
    for (mode, M, N, Kd), cfg in K._TUNED.items():
        e = ents.get((mode, M, N, Kd), {"mode": mode, "M": M, "N": N, "Kd": Kd})
        e["cfg"] = list(cfg)
        ents[(mode, M, N, Kd)] = e
    for pk, (dcfg, wcfg) in K._TUNED_PAIR.items():
        e = ents.get(("pair",) + pk, {"mode": "pair", "M": pk[0], "N": pk[1], "Kd": pk[2], "wgrad": list(pk[3:])})
        e["cfg"], e["wcfg"], e["ingraph"] = list(dcfg), list(wcfg), True
        ents[("pair",) + pk] = e
    out = {"model": old.get("model", "resnet34"), "batch": old.get("batch", B), "arch": "gfx950",
           "entries": sorted(ents.values(), key=lambda e: (e["mode"], -e["M"]))}
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({"final_ms": round(base, 4), "wall_s": round(time.time() - t_start, 1)}), flush=True)


if __name__ == "__main__":
    main()
