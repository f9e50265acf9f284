"""Elastic-parallelism driver (north-star config 4: VGG-16 / CIFAR-100 at P = 2 -> 4 -> 8).

Starts the single-node server with N GPU workers and a scripted scheduler policy
(``--policy scripted:2,4,8``: the reference's scheduler decides parallelism between
epochs, ml/pkg/scheduler/policy.go:50-94; here the sequence is fixed so runs are
reproducible — use ``--policy throughput`` for the reference policy), uploads a
synthetic dataset of the function's shape and runs an elastic (non-static) job.
Parallelism above N is clamped to N (one worker per MI355X).

Reports per epoch: parallelism, wall seconds, train-task seconds, images/s, the
per-worker model checksums (every active worker must hold the same model) and the
validation accuracy, from the job's history and log.

    python tools/run_elastic.py --gpus 8 --function vgg16 --policy scripted:2,4,8 --epochs 3
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

FUNCS = {"vgg16": ("function_vgg16.py", "cifar100", 100), "resnet34": ("function_resnet34.py", "cifar10", 10),
         "resnet32": ("function_resnet32.py", "cifar10", 10)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--function", choices=sorted(FUNCS), default="vgg16")
    ap.add_argument("--policy", default="scripted:2,4,8")
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--k", type=int, default=-1)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--n-train", type=int, default=50000)
    ap.add_argument("--n-test", type=int, default=10000)
    ap.add_argument("--cpu", action="store_true", help="CPU workers (gloo) rehearsal")
    a = ap.parse_args()

    from kubeml_amd.api.types import TrainOptions, TrainRequest
    from kubeml_amd.client import KubemlClient
    from kubeml_amd.config import Config
    from kubeml_amd.control.server import KubeMLServer

    code, dsname, ncls = FUNCS[a.function]
    tmp = tempfile.mkdtemp(prefix="kubeml_elastic_")
    cfg = Config()
    cfg.store_dir = os.path.join(tmp, "store")
    first = int(a.policy.split(":", 1)[1].split(",")[0]) if a.policy.startswith("scripted:") else 2
    srv = KubeMLServer(cfg, n_workers=a.gpus, use_gpu=not a.cpu, task_timeout=3600, policy=a.policy).start(
        ports={k: 0 for k in ("controller", "scheduler", "ps", "storage", "metrics")})
    try:
        c = KubemlClient(srv.url())
        rng = np.random.default_rng(0)
        arrs = {"xtr": rng.integers(0, 256, (a.n_train, 32, 32, 3), dtype=np.uint8),
                "ytr": rng.integers(0, ncls, a.n_train).astype(np.int64),
                "xte": rng.integers(0, 256, (a.n_test, 32, 32, 3), dtype=np.uint8),
                "yte": rng.integers(0, ncls, a.n_test).astype(np.int64)}
        paths = {}
        for k, v in arrs.items():
            paths[k] = os.path.join(tmp, f"{k}.npy")
            np.save(paths[k], v)
        c.datasets.create(dsname, paths["xtr"], paths["ytr"], paths["xte"], paths["yte"])
        c.functions.create(a.function, os.path.join(ROOT, "examples", code))
        jid = c.networks.train(TrainRequest(batch_size=a.batch, epochs=a.epochs, dataset=dsname, lr=a.lr,
                                            function_name=a.function,
                                            options=TrainOptions(default_parallelism=first, static_parallelism=False,
                                                                 validate_every=1, k=a.k)))
        t0 = time.time()
        last = t0
        while c.tasks.status(jid)["state"] == "running":
            time.sleep(0.25)
            if time.time() - last > 30:
                print(f"[run_elastic] running {time.time() - t0:.0f}s", flush=True)
                last = time.time()
        st = c.tasks.status(jid)
        if st["state"] != "finished":
            print(c.logs(jid).decode()[-4000:], file=sys.stderr)
            sys.exit(1)
        h = c.histories.get(jid).data
        recs = [json.loads(l) for l in c.logs(jid).decode().splitlines() if l.startswith("{")]
        eps = [r for r in recs if r.get("msg") == "epoch finished"]
        cum = list(h.epoch_duration)
        wall = [cum[0]] + [cum[i] - cum[i - 1] for i in range(1, len(cum))]
        rows = []
        for i, e in enumerate(eps):
            ck = e.get("checksums") or {}
            ends = [v[1] for v in ck.values() if v and v[1] is not None]
            rows.append({"epoch": e["epoch"], "parallelism": e["parallelism"], "wall_s": round(wall[i], 3),
                         "train_task_s": round(float(e["seconds"]), 3),
                         "img_s": round(a.n_train / float(e["seconds"]), 1),
                         "workers_consistent": (max(ends) - min(ends) <= 1e-6 * max(1.0, abs(ends[0]))) if ends else None,
                         "accuracy": round(h.accuracy[i], 3) if i < len(h.accuracy) else None})
        print(json.dumps({"function": a.function, "policy": a.policy, "gpus": a.gpus, "K": a.k, "batch": a.batch,
                          "epochs": rows, "parallelism": h.parallelism}), flush=True)
    finally:
        srv.stop()


if __name__ == "__main__":
    main()
