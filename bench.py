"""Headline benchmark: ResNet-34 / CIFAR-10 data-parallel training throughput on MI355X.

Metric (BASELINE.json): whole-node images/sec + epoch time for torchvision-style
ResNet-34 (ImageNet stem, 1000-class head, as in the reference's
ml/experiments/kubeml/function_resnet34.py) on 32x32 CIFAR-10 images, per-worker
batch 256, SGD(lr, weight_decay=1e-4), synchronous gradient all-reduce every step
(north-star config 2: K=1), bf16 compute with fp32 master weights.

The step is the framework's own: :func:`kubeml_amd.engine.dp.make_train_step`, the
builder ``KubeModel.step`` uses on resident workers (forward, backward, fused SGD, one
hipGraph replay per step).  With N > 1 the gradient exchange is the measured comm plan
(``kubeml_amd/parallel/comm_plan.json``; default ``peer:shard:fp32``: the fp32 gradient is
reduce-scattered straight out of the peers' HBM over xGMI, each rank applies SGD to its 1/N
of the master inside that kernel, and the bf16 weights are all-gathered — all inside the
captured step).  At N = 1 no collective runs (``config.sync`` says so).

Data: synthetic CIFAR-10-shaped uint8 images resident in HBM (no network for the
real dataset); every step runs the full on-device augmentation (random crop 32/pad 4,
horizontal flip, normalise) — nothing is skipped inside the timed region.
Weights: random init of the real architecture (21.8 M parameters).

After the timed steps a real epoch is MEASURED (not derived): every rank trains
ceil(50000 / N / B) full batches of its shard, BN statistics are averaged over the
ranks, then the 10,000-image validation set is evaluated (sharded over the ranks),
the reference's epoch time definition (ml/pkg/train/job.go:222-231, 327).

Usage:
  python bench.py --gpus N --steps K --warmup W
    N > 1 without WORLD_SIZE in the environment: the script launches N ranks itself
    (torch.distributed.run, one process per GPU, RCCL over xGMI) before touching the GPU.
  python bench.py --gpus N --cpu-smoke   (gloo on CPU: proves the N-rank launch path)
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_IMG_S = 4900.0  # P=8, batch 256, E=40 derivation (upper end of 3.7k-4.9k)
BASELINE_EPOCH_S = 10.0  # ~10-13.5 s/epoch at P=8, batch 256
CIFAR_TRAIN = 50000
CIFAR_TEST = 10000
METRIC = "images/sec (whole node) + epoch time, ResNet-34 CIFAR-10 at 1/2/4/8 workers"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256, help="per-worker batch (reference batch 256)")
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--bucket-mb", type=float, default=0.0)
    ap.add_argument("--trace-loss", action="store_true", help="print the loss of every step (debug; syncs)")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--overlap", choices=["auto", "on", "off"], default="auto",
                    help="stage-split backward with overlapped all-reduce (auto: on when N>1)")
    ap.add_argument("--force-comm", action="store_true",
                    help="run the RCCL all-reduce path even with one rank (single-GPU rehearsal of dp>1)")
    ap.add_argument("--graph-comm", choices=["on", "off"], default="on",
                    help="capture the RCCL all-reduces inside the step's hipGraph (off: eager between segment graphs)")
    ap.add_argument("--no-epoch", action="store_true", help="skip the measured epoch after the timed steps")
    ap.add_argument("--comm-dtype", choices=["fp32", "bf16"], default="fp32",
                    help="gradient all-reduce precision (bf16 = compressed, half the xGMI bytes)")
    ap.add_argument("--comm-plan", default="auto",
                    help="gradient transport backend:schedule:wire[:blocks] (e.g. peer:end:bf16:256, "
                         "rccl:overlap:fp32); auto = kubeml_amd/parallel/comm_plan.json's measured choice")
    ap.add_argument("--comm-timing", type=int, default=20,
                    help="sample the in-graph gradient all-reduce time every N steps (0 = off)")
    ap.add_argument("--e2e", choices=["auto", "on", "off"], default="auto",
                    help="also run the epoch through the whole framework (server, worker, storage, kubeml "
                         "train; kubeml_amd/experiments/e2e.py) and report e2e_epoch_time_s (auto: N = 1)")
    ap.add_argument("--cpu-smoke", action="store_true", help="gloo/CPU rehearsal of the N-rank launch (tiny model)")
    ap.add_argument("--trace", default=None, help="write a Chrome trace (device compute/comm timeline) to this dir; "
                                                  "collectives then run outside the step graph")
    return ap.parse_args()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _visible_gpus():
    """GPUs this process may use, without touching HIP: the *_VISIBLE_DEVICES lists, else the
    KFD topology's GPU nodes (simd_count > 0).  None when neither can be read."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([d for d in v.split(",") if d.strip() != ""])
    base = "/sys/class/kfd/kfd/topology/nodes"
    try:
        n = 0
        for node in os.listdir(base):
            with open(os.path.join(base, node, "properties")) as f:
                props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
            n += int(props.get("simd_count", "0")) > 0
        return n
    except OSError:
        return None


def relaunch(args):
    """--gpus N > 1 outside torchrun: start N ranks as a child torch.distributed.run and exit
    with its code.  The parent never loads HIP: it counts GPUs from the visible-devices
    variables or the KFD topology (sysfs)."""
    if not args.cpu_smoke:
        have = _visible_gpus()
        if have is not None and have < args.gpus:
            print(f"bench.py: --gpus {args.gpus} requested but only {have} GPU(s) visible "
                  f"(HIP_VISIBLE_DEVICES={os.environ.get('HIP_VISIBLE_DEVICES', '<unset>')})", file=sys.stderr)
            sys.exit(2)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    sys.exit(subprocess.call(cmd, env=env))


def cpu_smoke(args, world, rank, json_out=None):
    """N gloo ranks on CPU: LeNet, gradient all-reduce every step, one JSON line."""
    import torch
    import torch.distributed as dist
    from kubeml_amd.models.lenet import LeNet
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(args.seed)
    model = LeNet()
    opt = torch.optim.SGD(model.parameters(), lr=args.lr, weight_decay=1e-4)
    g = torch.Generator().manual_seed(rank)
    B = 8
    for _ in range(args.warmup + args.steps):
        x = torch.rand(B, 1, 28, 28, generator=g)
        y = torch.randint(0, 10, (B,), generator=g)
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(model(x), y)
        loss.backward()
        if world > 1:
            flat = torch.cat([p.grad.reshape(-1) for p in model.parameters()])
            dist.all_reduce(flat)
            flat /= world
            off = 0
            for p in model.parameters():
                p.grad.copy_(flat[off:off + p.numel()].view_as(p))
                off += p.numel()
        opt.step()
    cs = torch.tensor([float(sum(p.double().abs().sum() for p in model.parameters()))], dtype=torch.float64)
    joined = torch.ones(1)
    in_sync = True
    if world > 1:
        lo, hi = cs.clone(), cs.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        dist.all_reduce(joined)
        in_sync = bool(float(hi - lo) <= 1e-9 * max(1.0, float(hi)))
    if rank == 0:
        print(json.dumps({"metric": "cpu-smoke (gloo launch rehearsal; not a performance number)", "value": None,
                          "unit": None, "n_gpus": 0, "ranks": world, "ranks_joined": int(joined.item()),
                          "ranks_in_sync": in_sync, "steps": args.steps, "warmup": args.warmup,
                          "config": {"model": "lenet5", "backend": "gloo"}}), file=json_out or sys.stdout, flush=True)
    if world > 1:
        dist.destroy_process_group()


def _claim_stdout():
    """Keep stdout for the ONE JSON line: native libraries (RCCL prints its version banner
    to fd 1 when a communicator is created) write to stderr instead.  Returns the stream
    the JSON line goes to."""
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        relaunch(args)
    json_out = _claim_stdout()
    if "WORLD_SIZE" in os.environ and world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    if args.cpu_smoke:
        return cpu_smoke(args, world, rank, json_out)

    import torch
    import torch.distributed as dist
    if args.trace:
        from kubeml_amd.utils import trace as _trace
        _trace.enable(True)
        _trace.set_process("bench", rank)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    comm = world > 1 or args.force_comm
    if comm:
        dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)

    from kubeml_amd.engine.dp import make_train_step
    from kubeml_amd.models.resnet import resnet34
    from kubeml_amd.nn import cross_entropy, flatten_module
    from kubeml_amd.ops import kernels as K
    from kubeml_amd.optim import SGD
    from kubeml_amd.parallel.comm import from_env
    from kubeml_amd.parallel.kavg import ModelAverager

    B = args.batch
    n_local = CIFAR_TRAIN // world          # split_minibatches gives every rank ~1/N of the docs
    # the 10,000-image test set split over the ranks exactly (the ranks' shares sum to 10,000)
    n_val = CIFAR_TEST // world + (rank < CIFAR_TEST % world)

    # synthetic CIFAR-10 shards resident in HBM (each rank its own shard)
    g = torch.Generator(device=dev).manual_seed(rank)
    data = torch.randint(0, 256, (n_local, 32, 32, 3), dtype=torch.uint8, device=dev, generator=g)
    labels = torch.randint(0, 10, (n_local,), dtype=torch.int64, device=dev, generator=g)
    vdata = torch.randint(0, 256, (n_val, 32, 32, 3), dtype=torch.uint8, device=dev, generator=g)
    vlabels = torch.randint(0, 10, (n_val,), dtype=torch.int64, device=dev, generator=g)
    ctr = torch.tensor([float(1000 + rank), 0.0, 0.0], dtype=torch.float32, device=dev)
    xbuf = torch.empty((B, 32, 32, 8), dtype=torch.bfloat16, device=dev)
    ybuf = torch.empty((B,), dtype=torch.int64, device=dev)

    torch.manual_seed(args.seed)  # identical init on every rank
    model = resnet34(num_classes=1000).to(dev)
    space = flatten_module(model)
    cm = from_env()
    averager = ModelAverager(model)
    if comm:
        averager.broadcast_(cm, 0)
    model.train()
    opt = SGD(model.parameters(), lr=args.lr, weight_decay=1e-4)

    overlap = args.overlap == "on" or (args.overlap == "auto" and comm)
    graph_comm = args.graph_comm == "on"
    plan = None
    if comm:
        from kubeml_amd.parallel.plan import choose_plan
        plan = choose_plan(world, space.grad.numel() * 4,
                           override=None if args.comm_plan == "auto" else args.comm_plan)
    step = make_train_step(
        model, space, opt, cross_entropy, xbuf, ybuf,
        pre=lambda: K.augment(data, labels, ctr, B, out=xbuf, labels_out=ybuf, train=True),
        advance=(ctr, B, n_local),   # data-counter advance, folded into the SGD launch
        world=world, use_graph=not args.no_graph, graph_comm=graph_comm, overlap=overlap,
        bucket_mb=args.bucket_mb, force_comm=args.force_comm, extra_state=[ctr],
        comm_dtype=torch.bfloat16 if args.comm_dtype == "bf16" else torch.float32,
        plan=plan, comm_timing=args.comm_timing if comm else 0)
    if comm:
        step.prime_comm()
    step.capture()
    loss = None
    for _ in range(args.warmup):
        loss = step()
    torch.cuda.synchronize()
    first_loss = float(loss.item()) if loss is not None else float("nan")

    def timed(fn):
        if comm:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        if comm:
            dist.barrier()
        dt = time.perf_counter() - t0
        if comm:
            t = torch.tensor([dt], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return dt, out

    def run_steps(n):
        l = None
        for i in range(n):
            l = step()
            if args.trace_loss and rank == 0:
                print(f"step {i} loss {float(l.item()):.4f} gnorm {float(space.grad.norm()):.3e}", flush=True)
        return l

    dt, loss = timed(lambda: run_steps(args.steps))
    last_loss = float(loss.item())
    if getattr(step, "peer", None) is not None:
        step.peer.check()          # a timed-out peer barrier poisons the sums: fail loudly
    space.sync_master()            # sharded update: complete the fp32 master (no-op otherwise)
    in_sync = None
    if comm:
        # every rank must hold identical weights after K all-reduced steps (checks that the
        # graph-replayed collectives really ran)
        cs = (space.master.double().abs().sum() + space.shadow.double().abs().sum()).view(1)
        lo, hi = cs.clone(), cs.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        in_sync = bool((hi - lo).abs().item() <= 1e-9 * max(1.0, abs(hi.item())))
    ms = dt / args.steps * 1e3
    img_s = B * world * args.steps / dt

    epoch = None
    if not args.no_epoch:
        epoch = measure_epoch(args, model, space, step, averager, cm, comm, world, dev, timed, n_local,
                              vdata, vlabels, ctr, xbuf, ybuf)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(img_s, 1),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(img_s / BASELINE_IMG_S, 3),
            "dtype": "bf16",
            "data": "synthetic (CIFAR-10-shaped uint8 in HBM, on-device crop/flip/normalize), random-init weights",
            "config": {"model": "resnet34 (torchvision, ImageNet stem, 1000-class head)", "global_batch": B * world,
                       "per_worker_batch": B, "seq_len": None, "image": "32x32x3", "parallelism": f"dp{world}",
                       "optimizer": "SGD lr=%g wd=1e-4" % args.lr,
                       "sync": ("gradient exchange every step (K=1): " + plan.tag()) if plan is not None
                       else "none (N=1: no collective in the step)",
                       "graph": not args.no_graph,
                       "overlap_segments": bool(comm and len(step.segments) > 1),
                       "graph_comm": bool(getattr(step, "graph_comm", graph_comm) and comm), "bucket_mb": args.bucket_mb,
                       "grad_comm_dtype": plan.wire if plan is not None else args.comm_dtype,
                       "comm_plan": plan.tag() if plan is not None else None,
                       "comm_plan_source": plan.source if plan is not None else None,
                       "comm_transport": (("peer" if getattr(step, "peer", None) is not None else "rccl")
                                          if comm else None),
                       "sgd_rider": getattr(step, "ride_plan", None),
                       "shard_riders": ({"slices": step.shard_ride["slices"],
                                         "carried_in_graph": len(step.shard_ride["state"]["taken"])}
                                        if getattr(step, "shard_ride", None) else None),
                       "step": "kubeml_amd.engine.dp.make_train_step"},
            "loss_first_last": [round(first_loss, 4), round(last_loss, 4)],
        }
        if epoch is not None:
            out.update(epoch)
            out["epoch_vs_baseline"] = round(BASELINE_EPOCH_S / epoch["epoch_time_s"], 2)
        if comm and step.comm_seconds() > 0:
            out["allreduce_ms"] = round(step.comm_seconds() * 1e3, 4)
        if in_sync is not None:
            out["ranks_in_sync"] = in_sync
            out["rccl_world"] = dist.get_world_size()
    if args.trace:
        from kubeml_amd.utils import trace as _trace
        _trace.flush(args.trace)
    if comm:
        dist.destroy_process_group()
    if rank == 0 and (args.e2e == "on" or (args.e2e == "auto" and world == 1 and not args.no_epoch)):
        # the same epoch through the framework's own path; this process's step is released first
        del step, model, space, opt, data, labels, vdata, vlabels
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        out.update(measure_e2e(img_s))
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)


def measure_e2e(bench_img_s):
    """Epoch time through the whole stack (kubeml_amd/experiments/e2e.py): 4 epochs of
    synthetic CIFAR-10 with validation every epoch; the steady epoch (epochs 3-4 of the job's
    cumulative epoch_duration: epoch 1 captures the train graph, epoch 2's wall holds the
    first validation's eval-graph capture) is the reference's time definition end to end;
    e2e_total_s is the job's whole cumulative time, warm-up included."""
    try:
        from kubeml_amd.experiments.e2e import run_e2e
        r = run_e2e(gpus=1, epochs=4, batch=256, k=1, validate=True,
                    progress=lambda m: print(m, file=sys.stderr, flush=True))
        return {"e2e_epoch_time_s": r["steady_epoch_s"], "e2e_first_epoch_s": r["first_epoch_s"],
                "e2e_warmup_epochs": r["warmup_epochs"], "e2e_total_s": r["total_s"],
                "e2e_epoch_wall_s": r["epoch_wall_s"], "e2e_train_task_img_s": r["steady_train_task_img_s"],
                "e2e_vs_bench_step_rate": round(r["steady_train_task_img_s"] / bench_img_s, 3),
                "e2e_vs_baseline": round(BASELINE_EPOCH_S / r["steady_epoch_s"], 2),
                "e2e_path": "kubeml train -f resnet34 --K 1 --batch 256 --validate-every 1 (server, worker, storage)"}
    except Exception as e:  # the headline number stands on its own; report why e2e is missing
        return {"e2e_epoch_time_s": None, "e2e_error": repr(e)[:300]}


def measure_epoch(args, model, space, step, averager, cm, comm, world, dev, timed, n_local, vdata, vlabels, ctr,
                  xbuf, ybuf):
    """One measured epoch: train over the shard, average BN statistics, validate."""
    import torch
    import torch.distributed as dist
    from kubeml_amd.nn import cross_entropy
    from kubeml_amd.ops import kernels as K
    B = args.batch
    steps = math.ceil(n_local / B)
    n_val = vdata.shape[0]
    vsteps = n_val // B                     # full validation batches ...
    vtail = n_val - vsteps * B              # ... and the partial last one (10,000 = 39 x 256 + 16)
    vctr = torch.zeros(3, dtype=torch.float32, device=dev)
    acc = torch.zeros(2, dtype=torch.float64, device=dev)    # [correct, count]
    xt = torch.empty((max(vtail, 1),) + tuple(xbuf.shape[1:]), dtype=xbuf.dtype, device=dev)
    yt = torch.empty((max(vtail, 1),), dtype=ybuf.dtype, device=dev)

    def val_batch(nb, xb, yb):
        K.augment(vdata, vlabels, vctr, nb, out=xb, labels_out=yb, pad=0, flip=False, train=False)
        K.advance_counter_(vctr, nb, n_val)
        with torch.no_grad():
            loss, correct = cross_entropy(model(xb), yb, return_correct=True)
        acc[0] += correct
        acc[1] += nb
    full = (lambda: val_batch(B, xbuf, ybuf))
    tail = (lambda: val_batch(vtail, xt, yt)) if vtail else None
    # eval forwards as graphs too (captured once, outside the timed region; BN in eval mode)
    model.eval()
    vgraph = tgraph = None
    if not args.no_graph:
        graphs = []
        for fn in (full, tail):
            if fn is None:
                graphs.append(None)
                continue
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                fn()
            torch.cuda.current_stream().wait_stream(s)
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                fn()
            graphs.append(gr)
        vgraph, tgraph = graphs
    model.train()
    acc.zero_()
    vctr.zero_()

    def train_epoch():
        for _ in range(steps):
            step()

    def validate():
        averager.average_buffers_(cm)          # K=1 semantics: BN statistics averaged over ranks
        model.eval()
        for _ in range(vsteps):
            if vgraph is not None:
                vgraph.replay()
            else:
                full()
        if tail is not None:
            if tgraph is not None:
                tgraph.replay()
            else:
                tail()
        model.train()
        if comm:
            dist.all_reduce(acc)

    t_train, _ = timed(train_epoch)
    t_val, _ = timed(validate)
    return {"epoch_time_s": round(t_train + t_val, 4), "epoch_train_s": round(t_train, 4),
            "epoch_val_s": round(t_val, 4), "epoch_steps_per_rank": steps, "val_images": int(acc[1].item()),
            "val_batches_per_rank": vsteps + (1 if vtail else 0),
            "epoch_measured": True}


if __name__ == "__main__":
    main()
