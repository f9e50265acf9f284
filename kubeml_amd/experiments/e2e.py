"""End-to-end framework measurement: the headline workload through the whole KubeML stack.

Starts the single-node server (controller, scheduler, PS, storage, metrics) with N GPU
workers, uploads a synthetic CIFAR-10-shaped dataset through the storage API, registers the
shipped ResNet-34 function (examples/function_resnet34.py) and runs

    kubeml train -f resnet34 -d cifar10 --K K --batch B --epochs E --parallelism N --static
                 [--validate-every 1]

Times come from the job's own history: ``epoch_duration`` is the cumulative wall time since
training start (reference ml/pkg/train/job.go:183, 327), so the per-epoch wall of epoch e
covers epoch e-1's validation and checkpoint plus epoch e's training — exactly the
reference's time definition.  The first epoch includes graph capture and warm-up; the
steady epoch is the mean of the later ones.  Used by ``tools/bench_e2e.py`` and by
``bench.py`` (its ``e2e_epoch_time_s``).
"""
from __future__ import annotations

import json
import os
import tempfile
import time
from typing import Optional

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run_e2e(gpus: int = 1, epochs: int = 3, batch: int = 256, k: int = 1, validate: bool = True,
            n_train: int = 50000, n_test: int = 10000, function: Optional[str] = None,
            trace_dir: Optional[str] = None, progress=None, timeout_s: float = 900.0) -> dict:
    from ..api.types import TrainOptions, TrainRequest
    from ..client import KubemlClient
    from ..config import Config
    from ..control.server import KubeMLServer
    function = function or os.path.join(ROOT, "examples", "function_resnet34.py")
    tmp = tempfile.mkdtemp(prefix="kubeml_e2e_")
    cfg = Config()
    cfg.store_dir = os.path.join(tmp, "store")
    t_start = time.time()
    srv = KubeMLServer(cfg, n_workers=gpus, use_gpu=True, task_timeout=1800).start(
        ports={p: 0 for p in ("controller", "scheduler", "ps", "storage", "metrics")})
    try:
        c = KubemlClient(srv.url())
        rng = np.random.default_rng(0)
        arrs = {"xtr": rng.integers(0, 256, (n_train, 32, 32, 3), dtype=np.uint8),
                "ytr": rng.integers(0, 10, n_train).astype(np.int64),
                "xte": rng.integers(0, 256, (n_test, 32, 32, 3), dtype=np.uint8),
                "yte": rng.integers(0, 10, n_test).astype(np.int64)}
        paths = {}
        for key, v in arrs.items():
            paths[key] = os.path.join(tmp, f"{key}.npy")
            np.save(paths[key], v)
        c.datasets.create("cifar10", paths["xtr"], paths["ytr"], paths["xte"], paths["yte"])
        c.functions.create("resnet34", function)
        t_submit = time.time()
        jid = c.networks.train(TrainRequest(batch_size=batch, epochs=epochs, dataset="cifar10", lr=0.01,
                                            function_name="resnet34",
                                            options=TrainOptions(default_parallelism=gpus, static_parallelism=True,
                                                                 validate_every=1 if validate else 0, k=k)))
        last = time.time()
        while c.tasks.status(jid)["state"] == "running":
            time.sleep(0.1)
            if time.time() - t_submit > timeout_s:
                raise TimeoutError(f"e2e job {jid} still running after {timeout_s:.0f} s")
            if progress is not None and time.time() - last > 30:
                progress(f"[e2e] running {time.time() - t_submit:.0f}s")
                last = time.time()
        st = c.tasks.status(jid)
        if st["state"] != "finished":
            raise RuntimeError(f"e2e job {jid} {st}: {c.logs(jid).decode()[-3000:]}")
        h = c.histories.get(jid).data
        cum = list(h.epoch_duration)
        per = [cum[0]] + [cum[i] - cum[i - 1] for i in range(1, len(cum))]
        logs = [json.loads(l) for l in c.logs(jid).decode().splitlines() if l.startswith("{")]
        ep = [l for l in logs if l.get("msg") == "epoch finished"]
        train_s = [float(l["seconds"]) for l in ep]
        # warm-up epochs: the first captures the train-step graph; the second's wall also holds
        # the first validation, which captures the eval-forward graph
        warm = 2 if len(per) >= 4 and validate else 1
        steady = per[warm:] or per
        steady_train = train_s[1:] or train_s
        return {
            "n_gpus": gpus, "K": k, "batch": batch, "epochs": epochs, "validate_every_epoch": validate,
            "epoch_wall_s": [round(x, 4) for x in per],
            "epoch_train_task_s": [round(x, 4) for x in train_s],
            "steady_epoch_s": round(sum(steady) / len(steady), 4),
            "steady_img_s": round(n_train / (sum(steady) / len(steady)), 1),
            "steady_train_task_s": round(sum(steady_train) / len(steady_train), 4),
            "steady_train_task_img_s": round(n_train / (sum(steady_train) / len(steady_train)), 1),
            "first_epoch_s": round(per[0], 4),
            "warmup_epochs": warm,
            "total_s": round(cum[-1], 4),      # the reference's epoch_duration[-1]
            "sync_mode": list(getattr(h, "sync_mode", [])),
            "sync_seconds": [l.get("sync_seconds") for l in ep],
            "grad_sync_rounds": [l.get("grad_sync_rounds") for l in ep],
            "train_loss": [round(x, 4) for x in h.train_loss],
            "setup_s": round(t_submit - t_start, 2),
        }
    finally:
        srv.stop()
        if trace_dir:
            import glob
            import shutil
            os.makedirs(trace_dir, exist_ok=True)
            for f in glob.glob(os.path.join(cfg.store_dir, "traces", "*.json")):
                shutil.copy(f, trace_dir)
        import shutil
        shutil.rmtree(tmp, ignore_errors=True)
