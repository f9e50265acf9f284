"""End-to-end framework benchmark: the headline workload through the whole KubeML stack.

Starts the single-node server (controller, scheduler, PS, storage, metrics) with N GPU
workers, uploads a synthetic CIFAR-10-shaped dataset (50,000 train / 10,000 test
uint8 32x32x3 images, random labels) through the storage API, registers the shipped
ResNet-34 function (examples/function_resnet34.py) and runs

    kubeml train -f resnet34 -d cifar10 --K 1 --batch 256 --epochs E --parallelism N --static
                 [--validate-every 1]

It reports, from the job's own history (``epoch_duration`` is cumulative wall time
since training start, reference ml/pkg/train/job.go:327) and log:
  * per-epoch wall time and images/s (epoch 1 includes graph capture and warm-up),
  * steady-state images/s = mean over epochs >= 2,
and compares with ``bench.py``'s step rate when given (--bench-img-s).

Usage: python tools/bench_e2e.py [--gpus N] [--epochs E] [--validate] [--bench-img-s X]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--epochs", type=int, default=4)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--k", type=int, default=1)
    ap.add_argument("--validate", action="store_true", help="validate every epoch (reference time definition)")
    ap.add_argument("--n-train", type=int, default=50000)
    ap.add_argument("--n-test", type=int, default=10000)
    ap.add_argument("--bench-img-s", type=float, default=None)
    ap.add_argument("--function", default=os.path.join(ROOT, "examples", "function_resnet34.py"))
    a = ap.parse_args()

    from kubeml_amd.api.types import TrainOptions, TrainRequest
    from kubeml_amd.client import KubemlClient
    from kubeml_amd.config import Config
    from kubeml_amd.control.server import KubeMLServer

    tmp = tempfile.mkdtemp(prefix="kubeml_e2e_")
    cfg = Config()
    cfg.store_dir = os.path.join(tmp, "store")
    srv = KubeMLServer(cfg, n_workers=a.gpus, use_gpu=True, task_timeout=1800).start(
        ports={k: 0 for k in ("controller", "scheduler", "ps", "storage", "metrics")})
    try:
        c = KubemlClient(srv.url())
        rng = np.random.default_rng(0)
        arrs = {"xtr": rng.integers(0, 256, (a.n_train, 32, 32, 3), dtype=np.uint8),
                "ytr": rng.integers(0, 10, a.n_train).astype(np.int64),
                "xte": rng.integers(0, 256, (a.n_test, 32, 32, 3), dtype=np.uint8),
                "yte": rng.integers(0, 10, a.n_test).astype(np.int64)}
        paths = {}
        for k, v in arrs.items():
            paths[k] = os.path.join(tmp, f"{k}.npy")
            np.save(paths[k], v)
        c.datasets.create("cifar10", paths["xtr"], paths["ytr"], paths["xte"], paths["yte"])
        c.functions.create("resnet34", a.function)
        t_submit = time.time()
        jid = c.networks.train(TrainRequest(batch_size=a.batch, epochs=a.epochs, dataset="cifar10", lr=0.01,
                                            function_name="resnet34",
                                            options=TrainOptions(default_parallelism=a.gpus, static_parallelism=True,
                                                                 validate_every=1 if a.validate else 0, k=a.k)))
        last = time.time()
        while c.tasks.status(jid)["state"] == "running":
            time.sleep(0.2)
            if time.time() - last > 30:
                print(f"[bench_e2e] running {time.time() - t_submit:.0f}s", flush=True)
                last = time.time()
        st = c.tasks.status(jid)
        if st["state"] != "finished":
            print(c.logs(jid).decode()[-4000:], file=sys.stderr)
            sys.exit(1)
        h = c.histories.get(jid).data
        cum = list(h.epoch_duration)
        per = [cum[0]] + [cum[i] - cum[i - 1] for i in range(1, len(cum))]
        logs = [json.loads(l) for l in c.logs(jid).decode().splitlines() if l.startswith("{")]
        ep = [l for l in logs if l.get("msg") == "epoch finished"]
        train_s = [float(l["seconds"]) for l in ep]
        img_epoch = [a.n_train / t for t in per]
        steady = img_epoch[1:] or img_epoch
        steady_train = [a.n_train / t for t in train_s[1:]] or [a.n_train / t for t in train_s]
        out = {"metric": "end-to-end kubeml train images/s (ResNet-34 CIFAR-10 shape, synthetic)",
               "n_gpus": a.gpus, "K": a.k, "batch": a.batch, "epochs": a.epochs, "validate_every_epoch": a.validate,
               "epoch_wall_s": [round(x, 4) for x in per], "epoch_train_task_s": [round(x, 4) for x in train_s],
               "img_s_per_epoch": [round(x, 1) for x in img_epoch],
               "steady_img_s": round(sum(steady) / len(steady), 1),
               "steady_train_task_img_s": round(sum(steady_train) / len(steady_train), 1),
               "sync_seconds": [l.get("sync_seconds") for l in ep],
               "grad_sync_rounds": [l.get("grad_sync_rounds") for l in ep],
               "train_loss": [round(x, 4) for x in h.train_loss]}
        if a.bench_img_s:
            out["vs_bench_step_rate"] = round(out["steady_train_task_img_s"] / a.bench_img_s, 3)
        print(json.dumps(out), flush=True)
    finally:
        srv.stop()


if __name__ == "__main__":
    main()
