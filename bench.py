"""Headline benchmark: ResNet-34 / CIFAR-10 data-parallel training throughput on MI355X.

Metric (BASELINE.json): whole-node images/sec (+ epoch time) for torchvision-style
ResNet-34 (ImageNet stem, 1000-class head, as in the reference's
ml/experiments/kubeml/function_resnet34.py) on 32x32 CIFAR-10 images, per-worker
batch 256, SGD(lr, weight_decay=1e-4), synchronous gradient all-reduce every step
(north-star config 2), bf16 compute with fp32 master weights.

Data: synthetic CIFAR-10-shaped uint8 images resident in HBM (no network for the
real dataset); every step runs the full on-device augmentation (random crop 32/pad 4,
horizontal flip, normalise) — nothing is skipped inside the timed region.
Weights: random init of the real architecture (21.8 M parameters).

Usage: python bench.py --gpus N --steps K --warmup W   (N>1 under torch.distributed.run)
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_IMG_S = 4900.0  # P=8, batch 256, E=40 derivation (upper end of 3.7k-4.9k)
CIFAR_TRAIN = 50000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256, help="per-worker batch (reference batch 256)")
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--bucket-mb", type=float, default=0.0)
    ap.add_argument("--trace-loss", action="store_true", help="print the loss of every step (debug; syncs)")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--segments", choices=["auto", "on", "off"], default="auto",
                    help="stage-split backward with overlapped all-reduce (auto: on when N>1)")
    ap.add_argument("--force-comm", action="store_true",
                    help="run the RCCL all-reduce path even with one rank (single-GPU rehearsal of dp>1)")
    ap.add_argument("--graph-comm", choices=["auto", "on", "off"], default="auto",
                    help="capture the overlapped all-reduces inside the step's hipGraph, one replay per step "
                         "(auto: on when N>1; KUBEML_GRAPH_COMM=0 forces off)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    comm = world > 1 or args.force_comm
    if comm:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)

    from kubeml_amd.engine.step import GraphedTrainStep
    from kubeml_amd.models.resnet import resnet34
    from kubeml_amd.nn import backward_loss, cross_entropy, flatten_module
    from kubeml_amd.ops import kernels as K
    from kubeml_amd.optim import SGD

    B = args.batch
    n_local = CIFAR_TRAIN // world

    # synthetic CIFAR-10 shard resident in HBM (each rank its own shard, like split_minibatches)
    g = torch.Generator(device=dev).manual_seed(rank)
    data = torch.randint(0, 256, (n_local, 32, 32, 3), dtype=torch.uint8, device=dev, generator=g)
    labels = torch.randint(0, 10, (n_local,), dtype=torch.int64, device=dev, generator=g)
    ctr = torch.tensor([float(1000 + rank), 0.0, 0.0], dtype=torch.float32, device=dev)
    xbuf = torch.empty((B, 32, 32, 8), dtype=torch.bfloat16, device=dev)
    ybuf = torch.empty((B,), dtype=torch.int64, device=dev)

    torch.manual_seed(args.seed)  # identical init on every rank
    model = resnet34(num_classes=1000).to(dev)
    space = flatten_module(model)
    if comm:
        dist.broadcast(space.master, 0)
        space.refresh_shadow()
    model.train()
    opt = SGD(model.parameters(), lr=args.lr, weight_decay=1e-4)
    opt.set_grad_scale(1.0 / world)

    def fwd_bwd():
        K.augment(data, labels, ctr, B, out=xbuf, labels_out=ybuf, train=True)
        space.zero_grad()
        loss = cross_entropy(model(xbuf), ybuf)
        backward_loss(loss)
        return loss

    def opt_step():
        opt.step()
        K.advance_counter_(ctr, B, n_local)

    use_seg = args.segments == "on" or (args.segments == "auto" and comm)
    graph_comm = use_seg and comm and os.environ.get("KUBEML_GRAPH_COMM", "1") != "0" and (
        args.graph_comm == "on" or (args.graph_comm == "auto" and world > 1))
    segs = seg_grads = None
    if use_seg:
        # backward in 3 graph segments; each segment's gradients are all-reduced on the
        # RCCL stream while the next segment computes (engine/staged.py)
        from kubeml_amd.engine.staged import StagedForwardBackward

        def pre():
            K.augment(data, labels, ctr, B, out=xbuf, labels_out=ybuf, train=True)
            space.zero_grad()
        staged = StagedForwardBackward(model.stages(), lambda out: cross_entropy(out, ybuf), lambda: xbuf, pre=pre)
        segs = [staged.segment(k) for k in range(staged.n_segments)]
        sp = model.stage_params()
        seg_grads = [[space.grad_view(sp[len(sp) - 1 - k])] for k in range(len(sp))]
    step = GraphedTrainStep(fwd_bwd, opt_step, [space.grad], use_graph=not args.no_graph, warmup=3,
                            bucket_mb=args.bucket_mb, segments=segs, segment_grads=seg_grads,
                            force_segments=use_seg, force_comm=args.force_comm, graph_comm=graph_comm)
    step.capture()
    for _ in range(args.warmup):
        loss = step()
    torch.cuda.synchronize()
    first_loss = float(loss.item())

    if comm:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step()
        if args.trace_loss and rank == 0:
            print(f"step {i} loss {float(loss.item()):.4f} gnorm {float(space.grad.norm()):.3e}", flush=True)
    torch.cuda.synchronize()
    if comm:
        dist.barrier()
    dt = time.perf_counter() - t0
    last_loss = float(loss.item())
    in_sync = None
    if comm:
        # every rank must hold identical weights after K all-reduced steps (checks that the
        # graph-replayed collectives really ran)
        cs = space.master.double().abs().sum().view(1)
        lo, hi = cs.clone(), cs.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        in_sync = bool((hi - lo).abs().item() <= 1e-9 * max(1.0, abs(hi.item())))
    if comm:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms = dt / args.steps * 1e3
    img_s = B * world * args.steps / dt
    if rank == 0:
        out = {
            "metric": "images/sec (whole node) + epoch time, ResNet-34 CIFAR-10 at 1/2/4/8 workers",
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
                       "optimizer": "SGD lr=%g wd=1e-4" % args.lr, "sync": "all-reduce every step (K=1)",
                       "graph": not args.no_graph, "overlap_segments": use_seg,
                       "graph_comm": graph_comm},
            "epoch_time_s": round(CIFAR_TRAIN / img_s, 3),
            "loss_first_last": [round(first_loss, 4), round(last_loss, 4)],
        }
        if in_sync is not None:
            out["ranks_in_sync"] = in_sync
        print(json.dumps(out), flush=True)
    if comm:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
