"""All-reduce microbenchmark over RCCL/xGMI: bus bandwidth vs
message size, fp32 and bf16, eager and hipGraph-captured.

    python tools/allreduce_bench.py                       # N = 1 (runs anywhere)
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        tools/allreduce_bench.py                          # whole node
    python tools/allreduce_bench.py --gpus 8              # self-launches the ranks

For each size: time of one all-reduce (median over --iters, max over ranks), algbw =
bytes / t and busbw = algbw * 2 (n - 1) / n (the per-link traffic of a ring; on 8
fully connected MI355X each GPU has 7 xGMI links of ~153 GB/s, so a single ring is
per-link bound — RCCL runs several channels to use them all; NCCL_MIN_NCHANNELS /
NCCL_ALGO / NCCL_PROTO can be swept through the environment).  The graph column is
the same all-reduce captured ``--graph-batch`` times into one hipGraph and replayed:
the launch-overhead-free latency the training step sees (its collectives are captured).

``--oneshot`` adds the one-shot peer-memory all-reduce (``kubeml_amd.parallel.oneshot``:
one hop over the fully connected xGMI mesh instead of a ring) for fp32 sizes up to
``--oneshot-mb``, eager and graph-captured, next to RCCL.

The framework's payloads are marked: ResNet-34 gradients (87.2 MB fp32 in 4 stage
segments of 0.93 / 4.5 / 27.3 / 54.5 MB), LeNet (0.18 MB), BN buffers (34 KB).  One JSON line per
size on rank 0, then a summary line.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MARKS = {"lenet grads": 178_000, "bn buffers (resnet34)": 34_000, "resnet34 stage stem+layer1": 925_952,
         "resnet34 stage layer2": 4_465_664, "resnet34 stage layer3": 27_289_600,
         "resnet34 stage layer4+fc": 54_509_472, "resnet34 all grads": 87_190_688}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--min-bytes", type=int, default=4096)
    ap.add_argument("--max-bytes", type=int, default=256 << 20)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--graph-batch", type=int, default=10)
    ap.add_argument("--dtypes", default="fp32,bf16")
    ap.add_argument("--cpu", action="store_true", help="gloo on CPU (rehearsal)")
    ap.add_argument("--oneshot", action="store_true",
                    help="also time the one-shot peer-memory all-reduce (kubeml_amd.parallel.oneshot) for fp32 "
                         "sizes up to --oneshot-mb")
    ap.add_argument("--oneshot-mb", type=int, default=8)
    a = ap.parse_args()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
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
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    if a.cpu:
        dev = torch.device("cpu")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    def tmax(x):
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    oneshot = None
    if a.oneshot and dev.type == "cuda" and world > 1:
        from kubeml_amd.parallel.oneshot import OneShotAllReduce
        oneshot = OneShotAllReduce(None, cap_bytes=a.oneshot_mb << 20, device=dev)

    sizes = []
    b = a.min_bytes
    while b <= a.max_bytes:
        sizes.append(b)
        b *= 4 if b < (1 << 20) else 2
    sizes = sorted(set(sizes + [v for v in MARKS.values() if a.min_bytes <= v <= a.max_bytes]))
    results = []
    for dt_name in a.dtypes.split(","):
        dt = {"fp32": torch.float32, "bf16": torch.bfloat16}[dt_name]
        es = torch.tensor([], dtype=dt).element_size()
        for nbytes in sizes:
            n = max(1, nbytes // es)
            x = torch.ones(n, dtype=dt, device=dev)
            for _ in range(a.warmup):
                dist.all_reduce(x)
            sync()
            ts = []
            for _ in range(a.iters):
                dist.barrier()
                sync()
                t0 = time.perf_counter()
                dist.all_reduce(x)
                sync()
                ts.append(time.perf_counter() - t0)
            ts.sort()
            t = tmax(ts[len(ts) // 2])
            tg = None
            if dev.type == "cuda" and a.graph_batch > 0:
                g = torch.cuda.CUDAGraph()
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    dist.all_reduce(x)
                torch.cuda.current_stream().wait_stream(s)
                sync()
                with torch.cuda.graph(g, capture_error_mode="thread_local"):
                    for _ in range(a.graph_batch):
                        dist.all_reduce(x)
                g.replay()
                sync()
                dist.barrier()
                t0 = time.perf_counter()
                for _ in range(3):
                    g.replay()
                sync()
                tg = tmax((time.perf_counter() - t0) / (3 * a.graph_batch))
            t1 = t1g = None
            if oneshot is not None and oneshot.supports(x):
                for _ in range(a.warmup):
                    oneshot.all_reduce_(x)
                sync()
                ts = []
                for _ in range(a.iters):
                    dist.barrier()
                    sync()
                    t0 = time.perf_counter()
                    oneshot.all_reduce_(x)
                    sync()
                    ts.append(time.perf_counter() - t0)
                ts.sort()
                t1 = tmax(ts[len(ts) // 2])
                g1 = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g1):
                    for _ in range(a.graph_batch):
                        oneshot.all_reduce_(x)
                g1.replay()
                sync()
                dist.barrier()
                t0 = time.perf_counter()
                for _ in range(3):
                    g1.replay()
                sync()
                t1g = tmax((time.perf_counter() - t0) / (3 * a.graph_batch))
            algbw = n * es / t / 1e9
            bus = algbw * (2 * (world - 1) / world if world > 1 else 1.0)
            mark = [k for k, v in MARKS.items() if v == nbytes]
            rec = {"dtype": dt_name, "bytes": n * es, "us": round(t * 1e6, 2),
                   "us_graph": round(tg * 1e6, 2) if tg else None, "algbw_GBs": round(algbw, 2),
                   "busbw_GBs": round(bus, 2), "world": world}
            if t1 is not None:
                rec["oneshot_us"] = round(t1 * 1e6, 2)
                rec["oneshot_us_graph"] = round(t1g * 1e6, 2)
            if mark:
                rec["payload"] = mark[0]
            results.append(rec)
            if rank == 0:
                print(json.dumps(rec), flush=True)
    if rank == 0:
        big = [r for r in results if r["bytes"] >= (64 << 20)]
        print(json.dumps({"summary": True, "world": world, "backend": "gloo" if a.cpu else "nccl(rccl)",
                          "peak_busbw_GBs": max((r["busbw_GBs"] for r in results), default=None),
                          "busbw_ge64MB_GBs": max((r["busbw_GBs"] for r in big), default=None),
                          "small_latency_us": min((r["us"] for r in results), default=None),
                          "small_latency_graph_us": min((r["us_graph"] for r in results if r["us_graph"]), default=None),
                          "env": {k: v for k, v in os.environ.items() if k.startswith(("NCCL_", "RCCL_"))}}),
              flush=True)
    if oneshot is not None:
        if oneshot.errors():
            print(json.dumps({"oneshot_spin_giveups": oneshot.errors()}), flush=True)
        oneshot.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
