"""KubeModel — the user model API (reference python/kubeml/kubeml/network.py:29-476).

Same surface and semantics: subclass it, implement ``configure_optimizers``, ``init``,
``train(batch, idx) -> float``, ``validate(batch, idx) -> (accuracy, loss)`` and
``infer(data)``; the runtime calls ``start()`` with the task of the invocation
(``init`` / ``train`` / ``val`` / ``infer``).

What changed underneath (MI355X-first):
* a worker is a resident process bound to one MI355X; the network and its optimizer
  live in HBM across invocations of the same job (no reload from a tensor store);
* the K-AVG sync between intervals is an RCCL all-reduce of the flat parameter buffer
  (+ packed BN statistics) inside the worker group instead of "save to Redis, POST
  /next, wait for the Go merger, reload" (network.py:289-306, 395-461);
* ``configure_optimizers`` may return a stock ``torch.optim.SGD/Adam/AdamW``; on the GPU
  it is transparently replaced by the fused single-launch HIP optimizer with the same
  hyper-parameters (:func:`kubeml_amd.optim.from_torch`);
* ``self.step(x, y)`` is an optional helper that runs forward / loss / backward /
  optimizer as one hipGraph replay for static-shape batches.
"""
from __future__ import annotations

import logging
import os
from abc import ABC
from typing import Any, Callable, Dict, Iterable, List, Sequence, Tuple, Union

import numpy as np
import torch
import torch.nn as nn
from torch.utils.data import DataLoader

from ..api.errors import DataError, InvalidFormatError, KubeMLException, MergeError
from ..parallel.comm import LocalComm
from ..parallel.kavg import ModelAverager
from ..utils import fault, trace
from .context import current_task
from .dataset import KubeDataset, _KubeArgs
from .util import get_gpu, get_subset_period, max_rounds, split_minibatches


def _same_but_lr(a, b) -> bool:
    if type(a) is not type(b) or len(a.param_groups) != len(b.param_groups):
        return False
    for ga, gb in zip(a.param_groups, b.param_groups):
        if [id(p) for p in ga["params"]] != [id(p) for p in gb["params"]]:
            return False
        for k, v in ga.items():
            if k not in ("params", "lr", "initial_lr") and gb.get(k) != v:
                return False
    return True


class KubeModel(ABC):

    def __init__(self, network: nn.Module, dataset: KubeDataset, gpu: bool = False):
        self._network = network
        self._dataset = dataset
        self.platform = "gpu" if gpu else "cpu"
        self.device = None
        self.args = None
        self.logger = logging.getLogger("kubeml.function")
        self.lr = None
        self.batch_size = None
        self.task = None
        self.optimizer = None
        self.epoch = None
        self._averager = ModelAverager(network)
        self._graphed = None
        self._flat = None
        ctx = current_task()
        if ctx is not None:
            ctx.extra["kubemodel"] = self

    # ---- proxies to the torch module (network.py:55-89) ----------------------------
    def __call__(self, *args, **kwargs):
        return self._network(*args, **kwargs)

    def parameters(self):
        return self._network.parameters()

    def apply(self, fn: Callable[[nn.Module], None]):
        self._network.apply(fn)
        return self

    @property
    def network(self) -> nn.Module:
        return self._network

    # ---- task plumbing ----------------------------------------------------------------
    def _read_args(self):
        self.args = _KubeArgs.parse()
        self.lr = self.args.lr
        self.batch_size = self.args.batch_size
        self.task = self.args._task
        self.epoch = self.args.epoch

    def _comm(self):
        ctx = current_task()
        if ctx is None or ctx.comm is None:
            return LocalComm()
        return ctx.comm

    def _get_logger(self):
        self.logger = logging.getLogger(f"kubeml.fn.{self.args._job_id}.{self.args._func_id}")

    def start(self) -> Union[Dict[str, Any], List[str]]:
        """Run the task of the current invocation; returns the JSON-able result."""
        self._read_args()
        self._get_logger()
        if self.task == "init":
            return self._initialize()
        if self.task == "train":
            return {"loss": self._train()}
        if self.task == "val":
            acc, loss, length = self._validate()
            return {"loss": loss, "accuracy": acc, "length": length}
        if self.task == "infer":
            return {"predictions": self._infer()}
        raise KubeMLException(f"Task {self.task} not recognized", 400)

    # ---- init (network.py:174-189) --------------------------------------------------------
    def _initialize(self) -> List[str]:
        self._set_device()
        self.init()
        return [name for name in self._network.state_dict()]

    # ---- optimizer -------------------------------------------------------------------------
    def _config_optimizer(self):
        """``configure_optimizers`` runs at every train task, as in the reference where
        each invocation builds a fresh optimizer (user code may derive the LR from
        ``self.epoch``, function_resnet34.py:51-62).  On the resident GPU model an
        optimizer that only differs in LR is kept and retuned through its device LR
        scalar, so captured hipGraphs stay valid."""
        opt = self.configure_optimizers()
        if opt is not None and self.device is not None and self.device.type == "cuda":
            from ..optim import from_torch
            try:
                opt = from_torch(opt)
            except TypeError:
                pass
        old = self.optimizer
        if old is not None and opt is not None and _same_but_lr(old, opt):
            lr = opt.param_groups[0]["lr"]
            if hasattr(old, "set_lr"):
                old.set_lr(lr)
            else:
                for g in old.param_groups:
                    g["lr"] = lr
            opt = old
        elif old is not None and opt is not old:
            self._graphed = None  # graphs captured the old optimizer's step
        self.optimizer = opt
        if opt is not None and hasattr(opt, "set_grad_scale"):
            opt.set_grad_scale(1.0)

    def _reset_optimizer_state(self):
        """Reference behaviour at every K-AVG round (network.py:121-128)."""
        if self.optimizer is None:
            return
        if hasattr(self.optimizer, "reset_state"):
            self.optimizer.reset_state()
        else:
            from collections import defaultdict
            self.optimizer.state = defaultdict(dict)

    # ---- hooks -----------------------------------------------------------------------------
    def _on_train_start(self):
        self._set_device()
        self._restore()
        self._network.train()
        self._config_optimizer()

    def _restore(self):
        """Resume / recovery: load the job's last reference-model checkpoint (the
        rest of the workers receive it through the start-of-epoch broadcast)."""
        ctx = current_task()
        path = ctx.extra.get("restore") if ctx is not None else None
        if path and getattr(self, "_restored_from", None) != path:
            from ..store.ckpt import load_checkpoint
            load_checkpoint(self._network, path)
            self._restored_from = path

    def _on_train_end(self):
        pass

    def _on_iteration_start(self):
        self._reset_optimizer_state()

    def _on_iteration_end(self):
        pass

    def _batch_to_device(self, batch):
        if isinstance(batch, torch.Tensor):
            return batch.to(self.device, non_blocking=True)
        if isinstance(batch, tuple):
            return type(batch)(e.to(self.device, non_blocking=True) if isinstance(e, torch.Tensor) else e
                               for e in batch)
        if isinstance(batch, Sequence) and not isinstance(batch, (str, bytes)):
            return type(batch)([e.to(self.device, non_blocking=True) if isinstance(e, torch.Tensor) else e
                                for e in batch])
        return batch

    def _batches(self):
        """Minibatches of the loaded documents, in order (the reference's DataLoader
        is not shuffled, network.py:284)."""
        ds = self._dataset
        bs = self.batch_size
        if ds.has_batch_hook():
            n = len(ds.data)
            for i in range(0, n, bs):
                yield ds.collate_batch(ds.data[i:i + bs], ds.labels[i:i + bs])
            return
        loader = DataLoader(ds, batch_size=bs, pin_memory=self.device is not None and self.device.type == "cuda")
        yield from loader

    def _num_batches(self):
        return -(-len(self._dataset.data) // self.batch_size) if len(self._dataset.data) else 0

    # ---- train (network.py:252-310, K-AVG) ------------------------------------------------
    def _train(self) -> float:
        self._on_train_start()
        comm = self._comm()
        N, fid, K = self.args._N, self.args._func_id, self.args._K
        num_docs = self._dataset.num_docs
        # every worker starts the epoch from the same reference model
        with trace.span("broadcast"):
            self._averager.broadcast_(comm, 0)
        assigned = split_minibatches(range(num_docs), N)[fid]
        per = max(get_subset_period(K, self.batch_size, assigned), 1)
        intervals = list(range(assigned.start, assigned.stop, per))
        rounds = max_rounds(num_docs, N, K, self.batch_size) if comm.world > 1 else len(intervals)
        self.logger.debug("subsets per iteration %d, rounds %d", per, rounds)
        loss, num_iterations = 0.0, 0
        self.sync_seconds = 0.0
        for r in range(rounds):
            fault.point("round", rank=fid, epoch=self.epoch, round=r, task="train", job=self.args._job_id)
            participate = r < len(intervals)
            if participate:
                i = intervals[r]
                with trace.span("load", docs=per):
                    self._dataset._load_train_data(start=i, end=min(assigned.stop, i + per))
                num_iterations += self._num_batches()
                self._on_iteration_start()
                with trace.span("iteration", round=r):
                    for idx, batch in enumerate(self._batches()):
                        batch = self._batch_to_device(batch)
                        loss += float(self.train(batch, idx))
                self._on_iteration_end()
            try:
                import time as _t
                t0 = _t.perf_counter()
                with trace.span("average", round=r):
                    self._averager.average_(comm, participate)  # replaces save + /next + merge + reload
                self.sync_seconds += _t.perf_counter() - t0
            except Exception as e:  # the reference surfaces merge failures as MergeError
                raise MergeError(e)
        self._on_train_end()
        return loss / max(num_iterations, 1)

    # ---- validation (network.py:320-360) --------------------------------------------------
    def _on_validation_start(self):
        self._set_device()
        self._network.eval()

    def _validate(self) -> Tuple[float, float, int]:
        self._on_validation_start()
        comm = self._comm()
        assigned = split_minibatches(range(self._dataset.num_val_docs), self.args._N)[self.args._func_id]
        self._dataset._load_validation_data(start=assigned.start, end=assigned.stop)
        self._averager.broadcast_(comm, 0)
        acc, loss, nb = 0.0, 0.0, 0
        with torch.no_grad():
            for idx, batch in enumerate(self._batches()):
                batch = self._batch_to_device(batch)
                a, l = self.validate(batch, idx)
                acc += float(a)
                loss += float(l)
                nb += 1
        self._network.train()
        n = len(self._dataset.data) if self._dataset.data is not None else 0
        return acc / max(nb, 1), loss / max(nb, 1), n

    # ---- inference (defined properly; the reference's was non-functional) -----
    def _infer(self):
        ctx = current_task()
        data = ctx.data if ctx is not None else None
        if not data:
            raise DataError()
        self._set_device()
        if ctx is not None and ctx.checkpoint and getattr(self, "_infer_ckpt", None) != ctx.checkpoint:
            from ..store.ckpt import load_checkpoint
            load_checkpoint(self._network, ctx.checkpoint)
            self._infer_ckpt = ctx.checkpoint
        self._network.eval()
        with torch.no_grad():
            preds = self.infer(data)
        if isinstance(preds, torch.Tensor):
            t = preds.detach().cpu()
            return (t.float() if t.is_floating_point() else t).numpy().tolist()
        if isinstance(preds, np.ndarray):
            return preds.tolist()
        if isinstance(preds, list):
            return preds
        raise InvalidFormatError()

    # ---- device ---------------------------------------------------------------------------
    def _set_device(self):
        if self.platform == "cpu" or not torch.cuda.is_available():
            self.device = torch.device("cpu")
            return
        ctx = current_task()
        if ctx is not None and ctx.device is not None and getattr(ctx.device, "type", None) == "cuda":
            self.device = ctx.device
        else:
            self.device = torch.device("cuda", get_gpu(self.args._func_id if self.args is not None else 0))
        torch.cuda.set_device(self.device)
        if getattr(self._network, "_kml_flat", None) is None or self._network._kml_flat.device != self.device:
            self._network.to(self.device)
            from ..nn.flat import flatten_module
            self._flat = flatten_module(self._network, self.device)

    # ---- MI355X helper: graph-captured step --------------------------------------------------
    def step(self, x, y, loss_fn=None):
        """forward + loss + backward + optimizer step for one batch; on the GPU the first
        call for a given batch shape captures a hipGraph that later calls replay.
        Returns the (device) loss tensor."""
        from ..nn import backward_loss, cross_entropy
        loss_fn = loss_fn or cross_entropy
        key = (tuple(x.shape), tuple(y.shape), x.dtype)
        if self.device is None or self.device.type != "cuda" or os.environ.get("KUBEML_NO_GRAPH") == "1":
            self.optimizer.zero_grad()
            loss = loss_fn(self(x), y)
            loss.backward()
            self.optimizer.step()
            return loss
        g = self._graphed
        if g is None or g["key"] != key:
            from ..engine.step import GraphedTrainStep
            xs, ys = x.clone(), y.clone()

            def fb():
                self.optimizer.zero_grad()
                l = loss_fn(self(xs), ys)
                backward_loss(l)
                return l
            st = GraphedTrainStep(fb, self.optimizer.step, warmup=2)
            st.capture()
            g = self._graphed = {"key": key, "x": xs, "y": ys, "step": st}
        g["x"].copy_(x, non_blocking=True)
        g["y"].copy_(y, non_blocking=True)
        return g["step"]()

    # ---- user hooks (network.py:463-476) --------------------------------------------------
    def configure_optimizers(self) -> torch.optim.Optimizer:
        pass

    def init(self):
        pass

    def train(self, batch, batch_index: int) -> float:
        pass

    def validate(self, batch, batch_index: int) -> Tuple[float, float]:
        pass

    def infer(self, data: List[Any]) -> Union[torch.Tensor, np.ndarray, List[float]]:
        pass
