"""Training dynamics of the N>1 gradient exchange: bf16 wire vs fp32 wire vs ZeRO-1 shard.

VERDICT r3 asked for evidence that the gradient wire chosen for N > 1 does not cost accuracy:
the round-3 default rounded every gradient to bf16 twice (copy-in and the reduced chunk), while
the reference averages fp32 (ml/pkg/model/parallelSGD.go:26-54).  This trains ResNet-34
(ImageNet stem, 1000-class head, as function_resnet34.py) with P ranks sharing the one GPU of
the box (gloo bootstrap, the peer-memory collectives inside the captured step — exactly the
kernels an 8-GPU node runs over xGMI) on the learnable synthetic CIFAR-shaped task of
``tools/convergence_check.py``, each rank on its contiguous shard with its own augmentation
stream, global batch 256, SGD momentum 0.9 wd 1e-4.  Every plan is run for every seed; BN
running statistics are averaged over the ranks before each evaluation (K = 1 semantics, see
parallel/kavg.py average_buffers_).  The figure of merit is the mean of the last five
validation accuracies per run, then mean +- std over seeds.

    python tools/convergence_multirank.py [--ranks 2] [--seeds 1,2,3] [--steps 1500]
        [--plans peer:end:bf16:256,peer:end:fp32:256,peer:shard:fp32:256] [--out FILE]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def rank_main(rank, a, port, q):
    import torch
    import torch.distributed as dist
    import torch.nn.functional as F
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("gloo", rank=rank, world_size=a.ranks)
        from kubeml_amd.engine.dp import make_train_step
        from kubeml_amd.models.resnet import resnet34
        from kubeml_amd.nn import cross_entropy, flatten_module
        from kubeml_amd.ops import kernels as K
        from kubeml_amd.optim import SGD
        from kubeml_amd.parallel.comm import TorchComm
        from kubeml_amd.parallel.kavg import ModelAverager
        from kubeml_amd.parallel.plan import parse_plan
        from convergence_check import make_task
        comm = TorchComm(peer_data=True)
        P, B = a.ranks, a.batch // a.ranks
        results = []
        for seed in [int(s) for s in a.seeds.split(",")]:
            g = torch.Generator(device=dev).manual_seed(2024 + seed)
            common = torch.rand(1, 3, 8, 8, device=dev, generator=g) * 255.0
            base = a.mix * common + (1.0 - a.mix) * torch.rand(10, 3, 8, 8, device=dev, generator=g) * 255.0
            templates = F.interpolate(base, size=(38, 38), mode="bilinear", align_corners=False).permute(0, 2, 3, 1)
            xtr, ytr = make_task(a.n_train, g, dev, templates, a.noise, a.label_noise)
            xte, yte = make_task(a.n_test, g, dev, templates, a.noise, 0.0)
            lo, hi = rank * a.n_train // P, (rank + 1) * a.n_train // P
            xs, ys = xtr[lo:hi].contiguous(), ytr[lo:hi].contiguous()
            for spec in a.plans.split(","):
                torch.manual_seed(seed)
                model = resnet34(num_classes=1000).to(dev)
                space = flatten_module(model)
                model.train()
                opt = SGD(model.parameters(), lr=a.lr, momentum=0.9, weight_decay=1e-4)
                ctr = torch.tensor([float(100 * seed + rank), 0.0, 0.0], dtype=torch.float32, device=dev)
                xb = torch.empty((B, 32, 32, 8), dtype=torch.bfloat16, device=dev)
                yb = torch.empty((B,), dtype=torch.int64, device=dev)
                step = make_train_step(model, space, opt, cross_entropy, xb, yb,
                                       pre=lambda: K.augment(xs, ys, ctr, B, out=xb, labels_out=yb, train=True),
                                       advance=(ctr, B, xs.shape[0]), world=P, plan=parse_plan(spec),
                                       extra_state=[ctr])
                step.capture()
                averager = ModelAverager(model)
                evals, losses = [], []
                t0 = time.time()
                for s in range(a.steps):
                    loss = step()
                    if (s + 1) % a.eval_every == 0:
                        losses.append(float(loss))
                        space.sync_master()
                        averager.average_buffers_(comm)
                        if rank == 0:
                            model.eval()
                            vctr = torch.zeros(3, dtype=torch.float32, device=dev)
                            vx = torch.empty((a.eval_batch, 32, 32, 8), dtype=torch.bfloat16, device=dev)
                            vy = torch.empty((a.eval_batch,), dtype=torch.int64, device=dev)
                            correct = 0
                            with torch.no_grad():
                                for _ in range(a.n_test // a.eval_batch):
                                    K.augment(xte, yte, vctr, a.eval_batch, out=vx, labels_out=vy, pad=0,
                                              flip=False, train=False)
                                    K.advance_counter_(vctr, a.eval_batch, a.n_test)
                                    _, c = cross_entropy(model(vx), vy, return_correct=True)
                                    correct += int(c)
                            model.train()
                            evals.append(100.0 * correct / (a.n_test // a.eval_batch * a.eval_batch))
                            print(json.dumps({"seed": seed, "plan": spec, "step": s + 1, "acc": round(evals[-1], 2),
                                              "loss": round(losses[-1], 4)}), flush=True)
                        dist.barrier()
                torch.cuda.synchronize()
                if step.peer is not None:
                    step.peer.check()
                    step.peer.close()
                if rank == 0:
                    tail = evals[-5:]
                    results.append({"seed": seed, "plan": spec, "evals": [round(e, 2) for e in evals],
                                    "last5_mean": round(sum(tail) / len(tail), 3), "train_loss": losses,
                                    "wall_s": round(time.time() - t0, 1)})
                del step, model, space, opt
                dist.barrier()
        q.put((rank, results, None))
    except Exception as e:
        import traceback
        q.put((rank, None, repr(e) + traceback.format_exc()[-3000:]))
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--seeds", default="1,2,3")
    ap.add_argument("--plans", default="peer:end:bf16:256,peer:end:fp32:256,peer:shard:fp32:256")
    ap.add_argument("--steps", type=int, default=1500)
    ap.add_argument("--eval-every", type=int, default=100)
    ap.add_argument("--batch", type=int, default=256, help="global batch (split over the ranks)")
    ap.add_argument("--eval-batch", type=int, default=256)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--n-train", type=int, default=25600)
    ap.add_argument("--n-test", type=int, default=5120)
    ap.add_argument("--noise", type=float, default=70.0)
    ap.add_argument("--mix", type=float, default=0.75)
    ap.add_argument("--label-noise", type=float, default=0.2)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "convergence_multirank.json"))
    a = ap.parse_args()
    import torch.multiprocessing as mp
    from kubeml_amd.runtime.pool import free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=rank_main, args=(r, a, port, q)) for r in range(a.ranks)]
    for p in ps:
        p.start()
    got = [q.get(timeout=3600) for _ in ps]
    for p in ps:
        p.join(60)
    for rank, res, exc in got:
        if exc is not None:
            print(f"rank {rank} failed: {exc}", file=sys.stderr)
            sys.exit(1)
    runs = next(res for rank, res, _ in got if rank == 0)
    summary = {}
    for spec in a.plans.split(","):
        v = [r["last5_mean"] for r in runs if r["plan"] == spec]
        summary[spec] = {"mean_last5_acc": round(statistics.mean(v), 3),
                         "std_over_seeds": round(statistics.stdev(v), 3) if len(v) > 1 else 0.0, "per_seed": v}
    ref = summary.get("peer:end:fp32:256")
    if ref:
        for spec, s in summary.items():
            s["gap_vs_fp32_wire"] = round(s["mean_last5_acc"] - ref["mean_last5_acc"], 3)
    out = {"what": "P ranks on one GPU (gloo bootstrap, peer-memory collectives in the captured step), ResNet-34, "
                   "synthetic learnable CIFAR-shaped task (tools/convergence_check.py make_task)",
           "ranks": a.ranks, "global_batch": a.batch, "steps": a.steps, "eval_every": a.eval_every,
           "optimizer": f"SGD lr={a.lr} momentum 0.9 wd 1e-4", "summary": summary, "runs": runs}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(summary), flush=True)


if __name__ == "__main__":
    main()
