"""The data-parallel step with 2 and 4 ranks sharing the one GPU of the test box.

Each rank is its own process with its own HIP context, bootstrapped over gloo; the gradient
collectives are the peer-memory kernels (csrc/kernels/comm.hip), which map the other ranks'
HBM exactly as they would across xGMI — only the link differs.  RCCL itself refuses two
ranks on one device, which is why the peer data plane is the one exercised here.

For every comm plan (all-reduce at the end of the step, fp32 and bf16 wire; ZeRO-1 shard):
  * ``make_train_step`` captures the step with the collectives inside the hipGraph (warm-up
    local, state restored) and replays it;
  * after the first replay the update equals a single process that computes every rank's
    gradient on the same kernels, sums them in rank order and applies the optimizer with 1/P
    (fp32 wire and shard: rel <= 1e-5; bf16 wire: the bf16 rounding, rel < 1e-2);
  * after several replays every rank holds bit-identical weights (master and bf16 shadow).
Reference: the job's merge of the functions' models, ml/pkg/model/model.go:249-302 and
ml/pkg/model/parallelSGD.go:26-54 (fp32 sum, then average).
"""
import hashlib
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

B = 32


def _digest(t):
    return hashlib.sha1(t.detach().contiguous().view(torch.uint8).cpu().numpy().tobytes()).hexdigest()


def _batches(rank, steps, dev):
    g = torch.Generator(device=dev).manual_seed(100 + rank)
    xs = torch.randn(steps, B, 32, 32, 8, device=dev, generator=g).to(torch.bfloat16)
    xs[..., 3:] = 0
    ys = torch.randint(0, 10, (steps, B), device=dev, generator=g)
    return xs, ys


def _model(dev, opt_kind):
    from kubeml_amd.models.resnet import resnet18
    from kubeml_amd.nn import flatten_module
    from kubeml_amd.optim import SGD, AdamW
    torch.manual_seed(0)
    m = resnet18(10).to(dev)
    m.train()
    sp = flatten_module(m)
    if opt_kind == "adamw":
        opt = AdamW(m.parameters(), lr=1e-3, weight_decay=1e-2)
    elif opt_kind == "sgdm":
        opt = SGD(m.parameters(), lr=1e-2, momentum=0.9, weight_decay=1e-4)
    else:
        opt = SGD(m.parameters(), lr=1e-2, weight_decay=1e-4)
    return m, sp, opt


def _reference_updates(world, dev, opt_kind, steps):
    """Master change after ``steps`` data-parallel steps in ONE process: every step sums every
    rank's gradient (its own batch of that step, the current weights) in rank order and applies
    the optimizer with grad scale 1/P — what the multi-rank step must reproduce step after step
    (the ZeRO-1 plans included: a rank reads the fp32 master of BN / bias parameters it does
    not own)."""
    from kubeml_amd.nn import backward_loss, cross_entropy
    m, sp, opt = _model(dev, opt_kind)
    w0 = sp.master.clone()
    data = [_batches(r, steps, dev) for r in range(world)]
    for k in range(steps):
        gsum = None
        for r in range(world):
            xs, ys = data[r]
            sp.zero_grad()
            loss = cross_entropy(m(xs[k]), ys[k])
            backward_loss(loss)
            sp.finish_grads()
            g = sp.grad.clone()
            gsum = g if gsum is None else gsum + g
        sp.grad.copy_(gsum)
        opt.set_grad_scale(1.0 / world)
        opt.step()
    torch.cuda.synchronize()
    return sp.master - w0


def _reference_update(world, dev, opt_kind):
    """One update from the initial model: every rank's gradient on the same kernels (eager),
    summed in rank order, optimizer with grad scale 1/P."""
    from kubeml_amd.nn import backward_loss, cross_entropy
    m, sp, opt = _model(dev, opt_kind)
    w0 = sp.master.clone()
    gsum = None
    for r in range(world):
        xs, ys = _batches(r, 1, dev)
        sp.zero_grad()
        loss = cross_entropy(m(xs[0]), ys[0])
        backward_loss(loss)
        sp.finish_grads()
        g = sp.grad.clone()
        gsum = g if gsum is None else gsum + g
    sp.grad.copy_(gsum)
    opt.set_grad_scale(1.0 / world)
    opt.step()
    torch.cuda.synchronize()
    return sp.master - w0


def _rank_main(rank, world, port, q, cases):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    out = {}
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from kubeml_amd.engine.dp import make_train_step
        from kubeml_amd.nn import cross_entropy
        from kubeml_amd.parallel.plan import parse_plan
        for spec, opt_kind, steps in cases:
            m, sp, opt = _model(dev, opt_kind)
            xs, ys = _batches(rank, steps, dev)
            x = torch.empty_like(xs[0])
            y = torch.empty_like(ys[0])
            i = torch.zeros((), dtype=torch.int64, device=dev)

            def pre():
                x.copy_(xs.index_select(0, i.view(1)).squeeze(0))
                y.copy_(ys.index_select(0, i.view(1)).squeeze(0))

            def post():
                i.add_(1)
            w0 = sp.master.clone()
            step = make_train_step(m, sp, opt, cross_entropy, x, y, pre=pre, post=post, extra_state=[i],
                                   plan=parse_plan(spec), world=world)
            transport = type(step.peer).__name__ if step.peer is not None else None
            step.capture()
            step()
            torch.cuda.synchronize()
            sp.sync_master()
            upd1 = (sp.master - w0).cpu()
            for _ in range(steps - 1):
                step()
            torch.cuda.synchronize()
            sp.sync_master()
            torch.cuda.synchronize()
            if step.peer is not None:
                step.peer.check()
            digests = [_digest(sp.master), _digest(sp.shadow)]
            shadow_ok = bool(torch.equal(sp.shadow, sp.master.to(torch.bfloat16)))
            res = {"transport": transport, "digests": digests, "shadow_is_bf16_master": shadow_ok,
                   "finite": bool(torch.isfinite(sp.master).all())}
            ride = getattr(step, "shard_ride", None)
            if ride is not None:   # slices carried by the backward launches of the last replay's capture
                res["ride_slices"], res["ride_taken"] = ride["slices"], len(ride["state"]["taken"])
            if rank == 0:
                ref = _reference_update(world, dev, opt_kind).cpu()
                res["rel"] = float((upd1 - ref).norm() / ref.norm())
                if steps > 1:   # the whole trajectory, not only the first update
                    refn = _reference_updates(world, dev, opt_kind, steps).cpu()
                    upd = (sp.master - w0).cpu()
                    res["rel_final"] = float((upd - refn).norm() / refn.norm())
            out[spec + "/" + opt_kind] = res
            if step.peer is not None:
                step.peer.close()
            del step
            dist.barrier()
        q.put((rank, out, None))
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, None, repr(e) + traceback.format_exc()[-2500:]))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _spawn(world, cases):
    import torch.multiprocessing as mp
    from kubeml_amd.runtime.pool import free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_rank_main, args=(r, world, port, q, cases)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = [q.get(timeout=300) for _ in ps]
    finally:
        for p in ps:
            p.join(30)
            if p.is_alive():
                p.kill()
    for rank, out, exc in res:
        assert exc is None, (rank, exc)
    return {rank: out for rank, out, _ in res}


CASES = [("peer:end:fp32:256", "sgd", 4), ("peer:end:bf16:256", "sgd", 4), ("peer:shard:fp32:256", "sgd", 4),
         ("peer:shard:fp32:256", "sgdm", 3), ("peer:shard:fp32:256", "adamw", 3),
         ("peer:shardov:fp32:64", "sgd", 4), ("peer:shardov:fp32:64", "sgdm", 3),
         ("peer:shardride:fp32:256", "sgd", 4), ("peer:shardride:fp32:256", "sgdm", 3)]


def _check(world, res):
    for key in res[0]:
        spec = key.split("/")[0]
        rs = [res[r][key] for r in range(world)]
        want = "PeerShard" if ":shard" in spec else "PeerAllReduce"
        assert all(r["transport"] == want for r in rs), (key, [r["transport"] for r in rs])
        assert all(r["finite"] for r in rs), key
        # every rank holds bit-identical weights after the replays
        assert all(r["digests"] == rs[0]["digests"] for r in rs), (key, [r["digests"] for r in rs])
        assert all(r["shadow_is_bf16_master"] for r in rs), key
        if ":shardride:" in spec:   # every slice rode a backward launch (none ran on its own)
            assert all(r["ride_slices"] > 0 and r["ride_taken"] == r["ride_slices"] for r in rs), key
        rel = rs[0]["rel"]
        if ":bf16:" in spec:
            assert 0 < rel < 1e-2, (key, rel)
        else:
            assert rel <= 1e-5, (key, rel)
            if "rel_final" in rs[0]:
                assert rs[0]["rel_final"] <= 1e-4, (key, rs[0]["rel_final"])


def test_train_step_two_ranks_one_gpu():
    _check(2, _spawn(2, CASES))


def test_shard_riders_match_the_shard_step_bit_for_bit():
    """The riders apply the same recurrence in the same rank order as the end-of-backward shard
    step, so after several momentum steps (the first-step flag cleared between them) the weights
    are bit-identical.  Run back to back in fresh processes: plans that ran earlier in a process
    may have settled other per-process kernel routes (tools/diag/ride_vs_shard.py compares step
    by step)."""
    res = _spawn(2, [("peer:shard:fp32:256", "sgdm", 3), ("peer:shardride:fp32:256", "sgdm", 3)])
    for r in range(2):
        assert res[r]["peer:shardride:fp32:256/sgdm"]["digests"] == res[r]["peer:shard:fp32:256/sgdm"]["digests"]


def test_train_step_four_ranks_one_gpu():
    _check(4, _spawn(4, [c for c in CASES if c[1] == "sgd"]))


def test_staged_shard_plan_rides_the_backward_stages():
    """peer:shardov: the step is split at the model's backward stages and each stage runs its
    own reduce-scatter + SGD + all-gather on a side stream (ownership cut per stage)."""
    res = _spawn(2, [("peer:shardov:fp32:64", "sgd", 2)])
    r0 = res[0]["peer:shardov:fp32:64/sgd"]
    assert r0["transport"] == "PeerShard" and r0["rel"] <= 1e-5


def _rank_master_race(rank, world, port, q):
    """After a sharded step, rank 0 overwrites its own master chunk right after sync_master
    while rank 1 enters sync_master late: the gather's exit barrier must keep rank 0's write
    behind rank 1's read (gather_master had only an entry barrier)."""
    import time
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from kubeml_amd.engine.dp import make_train_step
        from kubeml_amd.nn import cross_entropy
        from kubeml_amd.parallel.plan import parse_plan
        m, sp, opt = _model(dev, "sgd")
        xs, ys = _batches(rank, 1, dev)
        x, y = xs[0].clone(), ys[0].clone()
        step = make_train_step(m, sp, opt, cross_entropy, x, y, plan=parse_plan("peer:shard:fp32:256"), world=world)
        assert type(step.peer).__name__ == "PeerShard"
        step.capture()
        step()
        torch.cuda.synchronize()
        sh = step.peer
        own = sp.master[sh.lo:sh.hi].clone()          # this rank's chunk is current before the gather
        torch.cuda.synchronize()
        dist.barrier()
        if rank == 1:
            time.sleep(0.3)                           # arrive late: rank 0 waits in the entry barrier
        sp.sync_master()
        if rank == 0:
            sp.master[sh.lo:sh.hi].fill_(12345.0)    # a local step right after the collective
        torch.cuda.synchronize()
        chunk0 = None
        if rank == 1:
            c0 = (0, sh.chunk) if sh.chunk <= sp.numel else (0, sp.numel)
            chunk0 = _digest(sp.master[c0[0]:min(c0[1], sp.numel)])
        mine = _digest(own)
        allv = [None] * world
        dist.all_gather_object(allv, (mine, chunk0))
        sh.check()
        q.put((rank, {"own": allv, "errors": sh.errors()}, None))
        sh.close()
    except Exception as e:
        import traceback
        q.put((rank, None, repr(e) + traceback.format_exc()[-2500:]))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_sync_master_exit_barrier_protects_late_readers():
    import torch.multiprocessing as mp
    from kubeml_amd.runtime.pool import free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_rank_master_race, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    try:
        res = [q.get(timeout=300) for _ in ps]
    finally:
        for p in ps:
            p.join(30)
            if p.is_alive():
                p.kill()
    for rank, out, exc in res:
        assert exc is None, (rank, exc)
    out = {rank: o for rank, o, _ in res}
    rank0_chunk_before, _ = out[1]["own"][0]
    _, rank1_saw = out[1]["own"][1]
    assert rank1_saw == rank0_chunk_before         # rank 1 gathered rank 0's chunk before the overwrite
    assert out[0]["errors"] == 0 and out[1]["errors"] == 0


def test_shard_selftest_failure_falls_back_to_allreduce():
    """A failing ZeRO-1 self-test (fault-injected on rank 1) must leave EVERY rank on the exact
    all-reduce plan — same update, identical ranks — instead of one rank diverging or hanging."""
    old = os.environ.get("KUBEML_FAULT")
    os.environ["KUBEML_FAULT"] = "raise:at=shard_selftest:rank=1"
    try:
        res = _spawn(2, [("peer:shard:fp32:256", "sgd", 3)])
    finally:
        if old is None:
            os.environ.pop("KUBEML_FAULT", None)
        else:
            os.environ["KUBEML_FAULT"] = old
    rs = [res[r]["peer:shard:fp32:256/sgd"] for r in range(2)]
    assert all(r["transport"] == "PeerAllReduce" for r in rs), [r["transport"] for r in rs]
    assert rs[0]["digests"] == rs[1]["digests"] and all(r["finite"] for r in rs)
    assert rs[0]["rel"] <= 1e-5, rs[0]["rel"]


def test_shard_rider_selftest_failure_falls_back_to_the_shard_step():
    """A failing shard-rider self-test (fault-injected on rank 1) must leave EVERY rank on the
    end-of-backward shard step: no rider armed on any host, same update, identical ranks."""
    old = os.environ.get("KUBEML_FAULT")
    os.environ["KUBEML_FAULT"] = "raise:at=rider_selftest:rank=1"
    try:
        res = _spawn(2, [("peer:shardride:fp32:256", "sgdm", 3)])
    finally:
        if old is None:
            os.environ.pop("KUBEML_FAULT", None)
        else:
            os.environ["KUBEML_FAULT"] = old
    rs = [res[r]["peer:shardride:fp32:256/sgdm"] for r in range(2)]
    assert all(r["transport"] == "PeerShard" for r in rs), [r["transport"] for r in rs]
    assert all("ride_slices" not in r for r in rs), rs          # the fallback step carries no riders
    assert rs[0]["digests"] == rs[1]["digests"] and all(r["finite"] for r in rs)
    assert rs[0]["rel"] <= 1e-5, rs[0]["rel"]
