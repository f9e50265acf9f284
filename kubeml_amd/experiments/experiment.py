"""Experiments that drive a running KubeML server like a user would (reference
ml/experiments/common/experiment.py:19-337).

* :class:`KubemlExperiment` — submit a static-parallelism train task (through the
  ``kubeml`` CLI exactly like the reference, ``--default-parallelism`` alias included,
  or through the Python client), poll ``task list --short`` until it leaves, fetch the
  history (``history get --network``), optionally collect system metrics meanwhile.
* :class:`TorchBaselineExperiment` — the comparison baseline.  The reference compared
  against TensorFlow ``MirroredStrategy`` (tflow/*.py, E2); TensorFlow is not part of
  this stack, so the baseline is stock PyTorch-ROCm data parallel training of the same
  network (``tools/stock_baseline.py``), recording per-epoch times the same way.

Results are saved as JSON / CSV (never pickles): one row per experiment with the
request fields flattened and the history arrays as lists, like the reference's
``to_dataframe``.
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import time
from abc import ABC, abstractmethod
from dataclasses import dataclass, field
from typing import List, Optional

from ..api.types import History, TrainRequest

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def get_title(req: TrainRequest) -> str:
    return (f"{req.model_type}-{req.dataset}-b{req.batch_size}-k{req.options.k}-p{req.options.default_parallelism}"
            f"-lr{req.lr}-e{req.epochs}")


def get_hash(title: str) -> str:
    return hashlib.sha256(title.encode()).hexdigest()[:16]


def retry(fn, tries: int = 5, backoff: float = 2.0, initial: float = 0.5):
    """Retry with exponential backoff (reference common/utils.py:83-120)."""
    wait = initial
    for i in range(tries):
        try:
            return fn()
        except Exception:
            if i == tries - 1:
                raise
            time.sleep(wait)
            wait *= backoff


class Experiment(ABC):
    def __init__(self, title: str):
        self.title = title

    @abstractmethod
    def run(self):
        ...

    @abstractmethod
    def to_row(self) -> dict:
        ...

    def save(self, path: str) -> str:
        os.makedirs(path, exist_ok=True)
        row = self.to_row()
        p = os.path.join(path, f"{row.get('id') or get_hash(self.title)}.json")
        with open(p, "w") as f:
            json.dump(row, f, indent=1)
        return p


class KubemlExperiment(Experiment):
    def __init__(self, title: str, request: TrainRequest, url: Optional[str] = None, use_cli: bool = True,
                 poll_s: float = 2.0, sampler=None):
        super().__init__(title)
        self.request = request
        self.url = url
        self.use_cli = use_cli
        self.poll_s = poll_s
        self.sampler = sampler
        self.network_id: Optional[str] = None
        self.history: Optional[History] = None

    # --- CLI plumbing (the reference shells out to the kubeml binary) ----------------
    def _cli(self, *args) -> str:
        cmd = [sys.executable, "-m", "kubeml_amd.cli"] + (["--url", self.url] if self.url else []) + list(args)
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, cwd=ROOT)
        if r.returncode != 0:
            raise RuntimeError(r.stderr.decode().strip() or f"kubeml {' '.join(args)} failed")
        return r.stdout.decode()

    def run_task(self) -> str:
        req = self.request
        if self.use_cli:
            args = ["train", "--function", req.function_name, "--dataset", req.dataset, "--epochs", str(req.epochs),
                    "--batch", str(req.batch_size), "--lr", str(req.lr),
                    "--default-parallelism", str(req.options.default_parallelism),
                    "--goal-accuracy", str(req.options.goal_accuracy), "--K", str(req.options.k),
                    "--validate-every", str(req.options.validate_every)]
            if req.options.static_parallelism:
                args.append("--static")
            return retry(lambda: self._cli(*args).strip().splitlines()[-1])
        from ..client import KubemlClient
        return KubemlClient(self.url).networks.train(req)

    def check_if_task_finished(self) -> bool:
        if self.use_cli:
            ids = retry(lambda: self._cli("task", "list", "--short")).split()
        else:
            from ..client import KubemlClient
            ids = [t.job.id for t in KubemlClient(self.url).tasks.list()]
        return self.network_id not in ids

    def get_model_history(self) -> History:
        if self.use_cli:
            return History.from_json(retry(lambda: self._cli("history", "get", "--network", self.network_id)))
        from ..client import KubemlClient
        return KubemlClient(self.url).histories.get(self.network_id)

    def run(self):
        self.network_id = self.run_task()
        if self.sampler is not None:
            self.sampler.start(self.network_id)
        try:
            while not self.check_if_task_finished():
                time.sleep(self.poll_s)
        finally:
            if self.sampler is not None:
                self.sampler.stop()
        self.history = self.get_model_history()
        return self.history

    def to_row(self) -> dict:
        h = self.history
        row = {"id": self.network_id, "hash": get_hash(self.title), "title": self.title}
        t = (h.task if h else self.request).to_dict()
        opts = t.pop("options")
        row.update(t)
        row.update(opts)
        if h is not None:
            row.update(h.data.to_dict())
        if self.sampler is not None:
            row["system"] = self.sampler.samples
        return row


class TorchBaselineExperiment(Experiment):
    """Stock PyTorch DP baseline of the same workload (replaces the TF baseline)."""

    def __init__(self, title: str, network: str = "resnet34", batch: int = 256, epochs: int = 1, gpus: int = 1,
                 steps: Optional[int] = None):
        super().__init__(title)
        self.network, self.batch, self.epochs, self.gpus, self.steps = network, batch, epochs, gpus, steps
        self.times: List[float] = []
        self.result: dict = {}

    def run(self):
        cmd = [sys.executable, os.path.join(ROOT, "tools", "stock_baseline.py"), "--batch", str(self.batch)]
        if self.steps:
            cmd += ["--steps", str(self.steps)]
        t0 = time.time()
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, cwd=ROOT)
        self.times.append(time.time() - t0)
        out = r.stdout.decode().strip().splitlines()
        try:
            self.result = json.loads(out[-1]) if out else {}
        except ValueError:
            self.result = {"raw": out[-5:]}
        if r.returncode != 0:
            self.result["error"] = r.stderr.decode()[-2000:]
        return self.result

    def to_row(self) -> dict:
        return {"id": get_hash(self.title), "title": self.title, "network": self.network, "batch": self.batch,
                "gpus": self.gpus, "times": self.times, **self.result}
