"""Comm/compute interference probe on ONE MI355X -> the data-parallel comm plan.

Question (profiles/launch_fusion_r2.md:86-91): the ResNet-34 backward is a chain of
~100 latency-bound launches, and any kernel resident on a second queue slows each of its
dispatches.  How much does an all-reduce running beside the backward cost, against running it
after the backward with the whole chip?

Measured here, all on the headline step (ResNet-34, batch 256, bf16, graph-captured):

1. ``base``      the step alone (what bench.py times at N=1).
2. ``stream``    the step with a side-queue HBM streamer forked at its start (a graph branch,
                 joined before the step ends) that moves the bytes one GPU moves in an N-rank
                 two-shot all-reduce of the fp32 (or bf16) gradient, 2 (N-1)/N * S, on
                 ``blocks`` workgroups; plus the streamer's duration alone.  This emulates an
                 overlapped collective of the real size, with the CU footprint of its grid cap.
   Two controls per row: the same streamer launched eagerly on a side stream next to each
   replay of the plain single-chain graph (queue contention without a graph branch), and the
   streamer appended serially after the step (no concurrency at all).
3. ``plans``     the real schedules at world 1 (a 1-rank group: the peer kernels run — copy-in,
                 reduce-scatter, all-gather — the link does not): ``peer:end``, ``peer:overlap``
                 at several block caps (in the graph, and ``/eager``: per-segment graph replays
                 with the collectives launched between them), and RCCL overlapped / end of step
                 (RCCL skips a 1-rank all-reduce, so those rows only price the graph structure).

The N-rank prediction per plan (documented model, the link is not measurable on one GPU):
    t_link(N)        = 2 (N-1)/N * S_wire / B_link   (B_link: --link-gbs, per-GPU aggregate read)
    end(N)           = t(peer:end, world 1) + t_link(N)
    overlap(N, b)    = t(peer:overlap b, world 1)
                       + rate(b) * max(0, min(t_link(N), hide) - d(b))    (longer side activity)
                       + max(0, t_link(N) - hide)                          (exposed tail)
    where rate(b) = (t_stream(b) - t_base) / d(b) is the measured slowdown per second of side
    activity and hide = the backward time after the first stage (--hide-frac of the step).
The plan with the smallest prediction wins per N; ties keep "end" (exact fp32, no second queue).
Writes the raw table (--out) and kubeml_amd/parallel/comm_plan.json (--plan-out).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=150)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--blocks", default="8,16,32,64,128")
    ap.add_argument("--link-gbs", type=float, default=300.0,
                    help="assumed per-GPU aggregate xGMI read bandwidth, GB/s (7 links; not measurable on 1 GPU)")
    ap.add_argument("--hide-frac", type=float, default=0.55,
                    help="fraction of the step after the first backward stage (the overlap window)")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "interference.json"))
    ap.add_argument("--plan-out", default=None)
    ap.add_argument("--skip-plans", action="store_true")
    ap.add_argument("--wires", default="fp32",
                    help="wire dtypes the plan choice may use (fp32 keeps the gradient sums fp32 end to end; "
                         "'fp32,bf16' also ranks the bf16 wire)")
    a = ap.parse_args()

    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
    from kubeml_amd.engine.dp import make_train_step
    from kubeml_amd.models.resnet import resnet34
    from kubeml_amd.nn import cross_entropy, flatten_module
    from kubeml_amd.ops import kernels as K
    from kubeml_amd.optim import SGD
    from kubeml_amd.parallel.peer import stream_copy
    from kubeml_amd.parallel.plan import parse_plan

    B = a.batch
    g = torch.Generator(device=dev).manual_seed(0)
    n_local = 50000
    data = torch.randint(0, 256, (n_local, 32, 32, 3), dtype=torch.uint8, device=dev, generator=g)
    labels = torch.randint(0, 10, (n_local,), dtype=torch.int64, device=dev, generator=g)
    torch.manual_seed(1234)
    model = resnet34(num_classes=1000).to(dev)
    space = flatten_module(model)
    model.train()
    opt = SGD(model.parameters(), lr=0.01, weight_decay=1e-4)
    S = space.grad.numel() * 4
    blocks_list = [int(b) for b in a.blocks.split(",")]
    rows = {"grad_bytes": S, "batch": B, "steps": a.steps, "link_gbs_assumed": a.link_gbs,
            "hide_frac": a.hide_frac}

    def build(pre_extra=None, post_extra=None, plan=None, graph_comm=True):
        ctr = torch.tensor([1000.0, 0.0, 0.0], dtype=torch.float32, device=dev)
        xbuf = torch.empty((B, 32, 32, 8), dtype=torch.bfloat16, device=dev)
        ybuf = torch.empty((B,), dtype=torch.int64, device=dev)

        def pre():
            K.augment(data, labels, ctr, B, out=xbuf, labels_out=ybuf, train=True)
            if pre_extra is not None:
                pre_extra()
        st = make_train_step(model, space, opt, cross_entropy, xbuf, ybuf, pre=pre, post=post_extra,
                             advance=(ctr, B, n_local), world=1, force_comm=plan is not None,
                             overlap=bool(plan is not None and plan.schedule == "overlap"), plan=plan,
                             extra_state=[ctr], graph_comm=graph_comm)
        st.capture()
        return st

    def time_step(st, n=a.steps, before=None):
        for _ in range(10):
            if before is not None:
                before()
            st()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            if before is not None:
                before()
            st()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    def log(**kw):
        print(json.dumps(kw), flush=True)

    snap = [t.detach().clone() for t in (space.state, space.shadow)]

    def restore():
        space.state.copy_(snap[0])
        space.shadow.copy_(snap[1])

    base = time_step(build())
    rows["base_ms"] = round(base, 4)
    log(base_ms=base)
    restore()

    # ---- 2. side-queue streamer of the N-rank per-GPU all-reduce bytes -----------------------
    src = torch.empty(S, dtype=torch.uint8, device=dev)
    dst = torch.empty(S, dtype=torch.uint8, device=dev)
    side = torch.cuda.Stream(dev)
    stream_rows = []
    for wire, wbytes in (("fp32", S), ("bf16", S // 2)):
        for N in (8,):
            nbytes = int(2 * (N - 1) / N * wbytes) // 16 * 16
            # the streamer copies nbytes: reads nbytes (as the links would deliver) and writes them
            passes = max(1, -(-nbytes // S))
            per = min(nbytes, S) // 16 * 16
            for b in blocks_list:
                # duration alone (graph of the streamer)
                gs = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gs):
                    stream_copy(src, dst, per, b, passes)
                gs.replay()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(50):
                    gs.replay()
                torch.cuda.synchronize()
                d = (time.perf_counter() - t0) / 50 * 1e3

                def fork(b=b, per=per, passes=passes):
                    cur = torch.cuda.current_stream(dev)
                    side.wait_stream(cur)
                    with torch.cuda.stream(side):
                        stream_copy(src, dst, per, b, passes)

                def join():
                    torch.cuda.current_stream(dev).wait_stream(side)
                t = time_step(build(pre_extra=fork, post_extra=join))
                restore()
                # the same streamer launched EAGERLY on a side stream next to each replay of the
                # plain (single-chain) step graph: hardware queue contention without a graph branch
                plain = build()

                def eager(b=b, per=per, passes=passes):
                    side.wait_stream(torch.cuda.current_stream(dev))
                    with torch.cuda.stream(side):
                        stream_copy(src, dst, per, b, passes)
                te = time_step(plain, before=eager)
                torch.cuda.synchronize()
                restore()
                # serial: the streamer after the step on the same stream (no concurrency)
                ts = time_step(build(post_extra=lambda b=b, per=per, passes=passes: stream_copy(src, dst, per, b,
                                                                                                 passes)))
                restore()
                r = {"wire": wire, "N": N, "bytes": nbytes, "blocks": b, "stream_alone_ms": round(d, 4),
                     "step_ms": round(t, 4), "slowdown_ms": round(t - base, 4),
                     "rate": round((t - base) / d, 4) if d > 0 else None,
                     "eager_side_step_ms": round(te, 4), "serial_step_ms": round(ts, 4)}
                stream_rows.append(r)
                log(**r)
    rows["stream"] = stream_rows

    # ---- 3. real schedules at world 1 ----------------------------------------------------------
    plan_rows = []
    if not a.skip_plans:
        specs = ["peer:end:fp32:256", "peer:end:bf16:256"]
        specs += [f"peer:overlap:{w}:{b}" for w in ("fp32", "bf16") for b in (16, 32, 64, 128)]
        specs += ["rccl:overlap:fp32", "rccl:end:fp32"]
        specs += [f"peer:overlap:{w}:{b}/eager" for w in ("fp32", "bf16") for b in (32, 128)]
        for spec in specs:
            plan = parse_plan(spec.split("/")[0], "probe")
            try:
                st = build(plan=plan, graph_comm=not spec.endswith("/eager"))
                t = time_step(st)
                cs = st.comm_seconds()
                r = {"plan": spec, "step_ms": round(t, 4), "vs_base_ms": round(t - base, 4)}
            except Exception as e:   # record, keep probing the others
                r = {"plan": spec, "error": repr(e)[:300]}
            restore()
            plan_rows.append(r)
            log(**r)
    rows["plans"] = plan_rows

    # ---- prediction per N ---------------------------------------------------------------------
    pm = {r["plan"]: r["step_ms"] for r in plan_rows if "step_ms" in r}
    choice, pred = {}, {}
    hide = a.hide_frac * base
    for N in (2, 4, 8):
        cands = {}
        for wire, wbytes in (("fp32", S), ("bf16", S // 2)):
            t_link = 2 * (N - 1) / N * wbytes / (a.link_gbs * 1e9) * 1e3
            e = pm.get(f"peer:end:{wire}:256")
            if e is not None:
                cands[f"peer:end:{wire}:256"] = e + t_link
            for b in (16, 32, 64, 128):
                o = pm.get(f"peer:overlap:{wire}:{b}")
                sr = [r for r in stream_rows if r["wire"] == wire and r["blocks"] == b]
                if o is None:
                    continue
                rate = sr[0]["rate"] if sr and sr[0]["rate"] is not None else 0.0
                d = sr[0]["stream_alone_ms"] if sr else 0.0
                extra = rate * max(0.0, min(t_link, hide) - d) + max(0.0, t_link - hide)
                cands[f"peer:overlap:{wire}:{b}"] = o + extra
        if cands:
            best = min(cands, key=lambda k: (round(cands[k], 3), 0 if ":end:" in k else 1))
            # exactness first: take bf16 only when it buys more than 3% of the step
            f32 = {k: v for k, v in cands.items() if ":fp32:" in k}
            if ":bf16:" in best and f32:
                bf = min(f32, key=f32.get)
                if cands[bf] <= cands[best] * 1.03:
                    best = bf
            allowed = {k: v for k, v in cands.items() if k.split(":")[2] in a.wires.split(",")}
            if allowed and best not in allowed:
                best = min(allowed, key=allowed.get)
            choice[str(N)] = best
            pred[str(N)] = {k: round(v, 4) for k, v in sorted(cands.items(), key=lambda kv: kv[1])}
    rows["predicted_ms"] = pred
    rows["choice"] = choice
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rows, f, indent=1)
    if a.plan_out:
        with open(a.plan_out, "w") as f:
            json.dump({"choice": choice, "predicted_ms": pred, "base_ms": rows["base_ms"],
                       "link_gbs_assumed": a.link_gbs, "wires_allowed": a.wires,
                       "source": "tools/interference_probe.py"}, f, indent=1)
    log(choice=choice)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
