"""Final weights of the end-of-backward shard step (peer:shard) and the shard riders
(peer:shardride) on packed ranks, each with the fp32 master gathered after every replay and only
after the first and last: max |difference| per flat parameter range (the riders' two stages and
the rest) against peer:shard with a gather every step.

    python tools/diag/ride_vs_shard.py [--world 2] [--steps 4] [--opt sgd]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def _rank(rank, world, port, q, steps, opt_kind):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import test_multirank_gpu as T
        from kubeml_amd.engine.dp import make_train_step
        from kubeml_amd.nn import cross_entropy
        from kubeml_amd.parallel.plan import parse_plan
        hist = {}
        ranges = None
        runs = [(spec, se) for spec in ("peer:shard:fp32:256", "peer:shardride:fp32:256") for se in (1, 0)]
        for spec, se in runs:
            m, sp, opt = T._model(dev, opt_kind)
            if ranges is None:
                rs = [sp.range_of(ps) for ps, _, _ in m.comm_ride_plan()]
                ranges = rs + [(rs[-1][1], sp.numel)]
            xs, ys = T._batches(rank, steps, dev)
            x, y = torch.empty_like(xs[0]), torch.empty_like(ys[0])
            i = torch.zeros((), dtype=torch.int64, device=dev)

            def pre():
                x.copy_(xs.index_select(0, i.view(1)).squeeze(0))
                y.copy_(ys.index_select(0, i.view(1)).squeeze(0))

            def post():
                i.add_(1)
            step = make_train_step(m, sp, opt, cross_entropy, x, y, pre=pre, post=post, extra_state=[i],
                                   plan=parse_plan(spec), world=world)
            step.capture()
            for k in range(steps):
                step()
                torch.cuda.synchronize()
                if se or k == 0 or k == steps - 1:
                    sp.sync_master()
                torch.cuda.synchronize()
            hist[(spec, se)] = (sp.master.clone().cpu(), sp.shadow.clone().cpu())
            step.peer.close()
            del step
            dist.barrier()
        ref = hist[runs[0]]
        out = []
        for key in runs[1:]:
            a = hist[key]
            row = []
            for lo, hi in ranges:
                row.append((float((a[0][lo:hi] - ref[0][lo:hi]).abs().max()),
                            float((a[1][lo:hi].float() - ref[1][lo:hi].float()).abs().max())))
            out.append((f"{key[0]} sync_every={key[1]}", row))
        q.put((rank, {"ranges": ranges, "diff": out}, None))
    except Exception as e:
        import traceback
        q.put((rank, None, repr(e) + traceback.format_exc()[-2000:]))
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--opt", default="sgd")
    a = ap.parse_args()
    import torch.multiprocessing as mp
    from kubeml_amd.runtime.pool import free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_rank, args=(r, a.world, port, q, a.steps, a.opt)) for r in range(a.world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(30)
    for rank, out, exc in sorted(res, key=lambda r: r[0]):
        if exc:
            print("rank", rank, "error", exc)
            continue
        print("rank", rank, "ranges", out["ranges"], "(final weights vs peer:shard with a sync every step)")
        for name, row in out["diff"]:
            print(f"  {name}: " + "  ".join(f"master {m:.3e} shadow {s:.3e}" for m, s in row), flush=True)


if __name__ == "__main__":
    main()
