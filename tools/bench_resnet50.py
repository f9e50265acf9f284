"""ResNet-50 training throughput on MI355X - north-star config 3 (ImageNet-shape synthetic
data, K-step local SGD).  Not the headline benchmark (bench.py: ResNet-34 / CIFAR-10, the
reference's published workload); the same engine on the large-image model.

* model: torchvision-layout resnet50 (Bottleneck [3, 4, 6, 3], 1000 classes), random init;
* data: synthetic uint8 224x224x3 images resident in HBM, on-device flip + normalise
  (no network for ImageNet);
* optimiser: SGD momentum 0.9, weight decay 1e-4; bf16 compute, fp32 master weights;
* sync: K-AVG, the reference's algorithm: K local steps per worker, then one RCCL
  all-reduce of the flat parameter buffer + BN statistics (parallel/kavg.py) and an
  optimiser-state reset; the timed region includes the averaging rounds.

    python tools/bench_resnet50.py [--gpus N] [--batch 128] [--K 8] [--steps 32] [--warmup 8]
                                   [--force-comm] [--async-kavg]

``--gpus N`` launches N ranks itself (torch.distributed.run, one process per GPU, RCCL over
xGMI).  ``--force-comm`` runs the averaging rounds through a 1-rank RCCL group at N = 1, so
the round's pack / all-reduce / finish kernels are inside the timed region even on one GPU.
``--async-kavg``: the overlapped staleness-1 average (parallel/kavg.py AsyncModelAverager).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--K", type=int, default=8, help="local steps per model average")
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--images", type=int, default=1024, help="synthetic images per worker")
    ap.add_argument("--size", type=int, default=224)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--force-comm", action="store_true", help="1-rank RCCL group: averaging rounds really run")
    ap.add_argument("--async-kavg", action="store_true", help="overlapped staleness-1 K-AVG")
    a = ap.parse_args()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        import socket
        import subprocess
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")))
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29571")
    if world > 1 or a.force_comm:
        dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)
    from kubeml_amd.engine.step import GraphedTrainStep
    from kubeml_amd.models.resnet import resnet50
    from kubeml_amd.nn import backward_loss, cross_entropy, flatten_module
    from kubeml_amd.ops import kernels as K
    from kubeml_amd.optim import SGD
    from kubeml_amd.parallel.comm import from_env
    from kubeml_amd.parallel.kavg import AsyncModelAverager, ModelAverager

    B, S, n = a.batch, a.size, a.images
    g = torch.Generator(device=dev).manual_seed(rank)
    data = torch.randint(0, 256, (n, S, S, 3), dtype=torch.uint8, device=dev, generator=g)
    labels = torch.randint(0, 1000, (n,), dtype=torch.int64, device=dev, generator=g)
    ctr = torch.tensor([float(11 + rank), 0.0, 0.0], dtype=torch.float32, device=dev)
    xbuf = torch.empty((B, S, S, 8), dtype=torch.bfloat16, device=dev)
    ybuf = torch.empty((B,), dtype=torch.int64, device=dev)
    torch.manual_seed(0)
    model = resnet50(1000).to(dev)
    space = flatten_module(model)
    model.train()
    opt = SGD(model.parameters(), lr=a.lr, momentum=0.9, weight_decay=1e-4)
    comm = from_env()
    avg = (AsyncModelAverager if a.async_kavg else ModelAverager)(model)
    # --force-comm at N = 1: the 1-rank RCCL group's rounds run in full (pack -> all-reduce ->
    # finish, divisor 1) instead of being skipped as a no-op
    avg.force = bool(a.force_comm)
    avg.broadcast_(comm, 0)

    def fwd_bwd():
        K.augment(data, labels, ctr, B, out=xbuf, labels_out=ybuf, pad=0, flip=True, train=True)
        space.zero_grad()
        loss = cross_entropy(model(xbuf), ybuf)
        backward_loss(loss)
        return loss

    def opt_step():
        opt.step()
        K.advance_counter_(ctr, B, n)

    step = GraphedTrainStep(fwd_bwd, opt_step, warmup=2)  # local steps: no gradient all-reduce
    step.capture()

    def run(nsteps):
        loss = None
        for i in range(nsteps):
            loss = step()
            if (i + 1) % a.K == 0:
                avg.average_(comm)   # K-AVG round (reference job.go:368-442)
                opt.reset_state()    # optimiser reset per round (reference network.py:121-128)
        return loss

    def settle():
        if a.async_kavg and avg.pending:
            avg.flush_(comm)         # the last overlapped round lands inside the timed region

    loss = run(a.warmup)
    torch.cuda.synchronize()
    first = float(loss)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loss = run(a.steps)
    settle()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms = dt / a.steps * 1e3
    img_s = B * world * a.steps / dt
    flop_img = 3 * 2 * 4.09e9 * (S / 224) ** 2  # fwd 4.09 GMAC/img at 224, train ~3x fwd
    if rank == 0:
        print(json.dumps({"metric": "ResNet-50 ImageNet-shape training images/s (K-AVG local SGD)",
                          "value": round(img_s, 1), "unit": "images/s", "n_gpus": world, "ms_per_step": round(ms, 3),
                          "per_worker_batch": B, "image": f"{S}x{S}x3", "K": a.K, "steps": a.steps,
                          "kavg": "async-staleness1" if a.async_kavg else "sync",
                          "rounds_in_timed_region": a.steps // a.K,
                          "comm": "rccl" if (world > 1 or a.force_comm) else "none (1 rank, rounds skipped)",
                          "dtype": "bf16", "optimizer": "SGD momentum 0.9 wd 1e-4",
                          "model_tflops": round(img_s * flop_img / 1e12, 1),
                          "loss_first_last": [round(first, 4), round(float(loss), 4)],
                          "data": "synthetic ImageNet-shaped uint8 in HBM, random-init weights"}), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
