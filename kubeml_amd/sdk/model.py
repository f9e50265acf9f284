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
  optimizer as one hipGraph replay (engine/dp.py; one graph per batch shape, captured
  without applying any update);
* K = 1 with an SGD-family optimizer and ``batch % 64 == 0`` (every K-round is exactly
  one minibatch): rounds in which every worker has data run as synchronous data
  parallelism — ``self.step`` all-reduces the gradients over the worker group inside
  the captured step, overlapped with backward.  Because the reference resets the
  optimizer state every round, one step from a common model followed by a weight
  average equals one step on the averaged gradient, so the result is the reference's
  K = 1 model average (python/kubeml/kubeml/network.py:276-310) at a fraction of the
  traffic; BN running statistics (a linear recurrence) are averaged once per epoch.
  Any round that cannot take this path uses the fused weight average;
* ``train()`` may return the loss as a device tensor: losses are accumulated on the
  device and read back once per task, not once per minibatch.
"""
from __future__ import annotations

import logging
import os
import time
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


def _progress():
    from ..runtime.worker import progress
    progress()


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
        self._graphs: Dict[tuple, dict] = {}       # train steps (engine/dp.py), by batch shape + comm
        self._eval_graphs: Dict[tuple, dict] = {}  # eval forwards (evaluate)
        self._shards: Dict[int, Any] = {}         # id(comm) -> PeerShard of this model's flat space
        self._flat = None
        self._sync_mode = "local"      # "grad": self.step all-reduces gradients (K=1 fast path)
        self._grad_comm = None
        self._synced_steps = 0
        self.sync_seconds = 0.0
        self._dry = False              # job warm-up (_warm): step / evaluate capture only
        self._dry_calls = 0            # step / evaluate calls seen in dry mode
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
        if self.task == "warm":
            return {"warmed": self._warm()}
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
            self._graphs.clear()  # graphs captured the old optimizer's step
            self._drop_shards()   # (a shard's fused update reads the optimizer's state too)
        self.optimizer = opt
        if opt is not None and hasattr(opt, "set_grad_scale"):
            opt.set_grad_scale(1.0)

    def _drop_shards(self):
        """Close the sharded-update transports of this model (collective: every worker runs the
        same function code, so every rank changes its optimizer at the same point).  Unmaps the
        peers' buffers and frees the barrier region instead of leaking them; a master left
        sharded by the last step is completed first."""
        if self._shards and self._flat is not None:
            self._flat.sync_master()
        for sh in list(self._shards.values()):
            try:
                sh.close()
            except Exception:
                try:
                    sh._release()
                except Exception:
                    pass
        self._shards.clear()
        if self._flat is not None and getattr(self._flat, "master_sync", None) is not None:
            self._flat.master_sync = None

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
            from ..runtime.worker import busy
            from ..store.ckpt import load_checkpoint
            with busy():
                load_checkpoint(self._network, path)
            self._restored_from = path

    def _on_train_end(self):
        pass

    def _persistent(self) -> bool:
        """TrainOptions.sync == "grad": optimizer state persists across K=1 rounds."""
        return self.args is not None and getattr(self.args, "_sync", "") == "grad"

    def _on_iteration_start(self):
        if not self._persistent():
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
        if ds._streaming is not None:
            st = ds._streamers[ds._streaming]
            for _ in range(self._num_batches()):
                x, y = st.next()
                yield ds.collate_device(x, y)
            return
        if ds.has_batch_hook():
            n = len(ds.data)
            for i in range(0, n, bs):
                yield ds.collate_batch(ds.data[i:i + bs], ds.labels[i:i + bs])
            return
        loader = DataLoader(ds, batch_size=bs, pin_memory=self.device is not None and self.device.type == "cuda")
        yield from loader

    def _num_batches(self):
        return -(-len(self._dataset.data) // self.batch_size) if len(self._dataset.data) else 0

    def _grad_sync_ok(self, comm, K) -> bool:
        """Can K=1 rounds run as synchronous gradient all-reduce (see module docstring)?"""
        if os.environ.get("KUBEML_GRAD_SYNC", "1") == "0":
            return False
        if K != 1 or comm.world <= 1 or self.device is None:
            return False
        if self.batch_size % 64 != 0:
            return False
        if self.device.type == "cuda" and getattr(comm, "group", "missing") == "missing":
            return False      # the captured collectives need a torch.distributed group
        if self._persistent():
            # persistent state: a gradient step on the averaged gradient IS the update of
            # synchronous data parallelism for any optimizer (Adam / AdamW moments included)
            return True
        return getattr(self.optimizer, "kind", None) == "sgd" or type(self.optimizer) is torch.optim.SGD

    # ---- train (network.py:252-310, K-AVG) ------------------------------------------------
    def _train(self) -> float:
        with trace.span("train_start"):
            self._on_train_start()
        comm = self._comm()
        N, fid, K = self.args._N, self.args._func_id, self.args._K
        num_docs = self._dataset.num_docs
        # every worker starts the epoch from the same reference model
        with trace.span("broadcast"):
            self._averager.broadcast_(comm, 0)
        ctx = current_task()
        if ctx is not None and os.environ.get("KUBEML_CHECKSUMS", "1") != "0":
            with trace.span("checksum"):
                ctx.extra["start_checksum"] = self.model_checksum()
        splits = split_minibatches(range(num_docs), N)
        assigned = splits[fid]
        per = max(get_subset_period(K, self.batch_size, assigned), 1)
        intervals = list(range(assigned.start, assigned.stop, per))
        rounds = max_rounds(num_docs, N, K, self.batch_size) if comm.world > 1 else len(intervals)
        # rounds in which EVERY worker has data (uneven shards differ by at most one doc)
        full_rounds = min(-(-len(sp) // max(get_subset_period(K, self.batch_size, sp), 1)) for sp in splits)
        grad_ok = self._grad_sync_ok(comm, K)
        # overlapped staleness-1 K-AVG (opt-in: class attribute ASYNC_KAVG or KUBEML_KAVG_ASYNC=1)
        use_async = (not grad_ok and comm.world > 1 and
                     (getattr(self, "ASYNC_KAVG", False) or os.environ.get("KUBEML_KAVG_ASYNC") == "1"))
        if use_async and getattr(self, "_async_averager", None) is None:
            from ..parallel.kavg import AsyncModelAverager
            self._async_averager = AsyncModelAverager(self._network)
        if grad_ok:
            self._grad_comm = comm
            self._prime_grad_sync()
        self.logger.debug("subsets per iteration %d, rounds %d, grad-sync %s", per, rounds, grad_ok)
        # every minibatch of this task queued on the pinned stream (GPU, batch-hook datasets)
        with trace.span("plan_stream"):
            self._dataset._plan_stream("train", [(i, min(assigned.stop, i + per)) for i in intervals],
                                       self.batch_size, self.device)
        loss_host, loss_dev, num_iterations = 0.0, None, 0
        self.sync_seconds = 0.0
        grad_rounds = 0
        try:
            for r in range(rounds):
                fault.point("round", rank=fid, epoch=self.epoch, round=r, task="train", job=self.args._job_id)
                _progress()
                if r == full_rounds and self._flat is not None:
                    self._flat.sync_master()   # sharded update -> local rounds read the whole master
                    if grad_ok and self._persistent():
                        self._sync_optimizer_state(comm)
                participate = r < len(intervals)
                self._sync_mode = "grad" if (grad_ok and r < full_rounds) else "local"
                self._synced_steps = 0
                nb = 0
                if participate:
                    i = intervals[r]
                    with trace.span("load", docs=per):
                        self._dataset._load_train_data(start=i, end=min(assigned.stop, i + per))
                    nb = self._num_batches()
                    num_iterations += nb
                    self._on_iteration_start()
                    with trace.span("iteration", round=r):
                        for idx, batch in enumerate(self._batches()):
                            _progress()
                            batch = self._batch_to_device(batch)
                            l = self.train(batch, idx)
                            if isinstance(l, torch.Tensor):
                                l = l.detach().reshape(()).float()
                                loss_dev = l.clone() if loss_dev is None else loss_dev.add_(l)
                            else:
                                loss_host += float(l)
                    self._on_iteration_end()
                if self._sync_mode == "grad" and self._synced_steps == nb == 1:
                    grad_rounds += 1      # weights already identical on every rank
                    continue
                try:
                    t0 = time.perf_counter()
                    with trace.span("average", round=r):
                        if use_async and r < full_rounds:
                            self._async_averager.average_(comm)          # overlapped with the next round
                        elif use_async:
                            self._async_averager.flush_(comm, participate)   # ragged tail: synchronous
                        else:
                            self._averager.average_(comm, participate)  # replaces save + /next + merge + reload
                    self.sync_seconds += time.perf_counter() - t0
                except Exception as e:  # the reference surfaces merge failures as MergeError
                    raise MergeError(e)
                if self.PEER_CHECK_EVERY and (r + 1) % self.PEER_CHECK_EVERY == 0:
                    comm.check()     # a timed-out peer collective stops the task within a few rounds
            if use_async and self._async_averager.pending:
                t0 = time.perf_counter()
                with trace.span("average_flush"):
                    self._async_averager.flush_(comm)          # every worker ends on the same model
                self.sync_seconds += time.perf_counter() - t0
            if self._flat is not None:
                self._flat.sync_master()       # collective over the shard group (no-op if current)
            if grad_rounds:
                # in-graph gradient all-reduce time (device stamps sampled by the step)
                cs = [g["step"].comm_seconds() for k, g in self._graphs.items() if k[5]]
                cs = [c for c in cs if c > 0]
                if cs:
                    self.sync_seconds += sum(cs) / len(cs) * grad_rounds
                t0 = time.perf_counter()
                with trace.span("average_buffers"):
                    self._averager.average_buffers_(comm)
                self.sync_seconds += time.perf_counter() - t0
        finally:
            self._sync_mode = "local"
            self._grad_comm = None
            self._dataset._stream_end()
        self._on_train_end()
        if loss_dev is not None:
            with trace.span("loss_sync"):          # waits for the queued steps to finish
                loss_host += float(loss_dev.item())
        self.grad_rounds = grad_rounds
        if ctx is not None and os.environ.get("KUBEML_CHECKSUMS", "1") != "0":
            ctx.extra["end_checksum"] = self.model_checksum()
        if ctx is not None:   # reported to the job driver with the task result (metrics)
            ctx.extra["sync_seconds"] = self.sync_seconds
            ctx.extra["grad_rounds"] = grad_rounds
            ctx.extra["sync_mode"] = ("grad-allreduce" if grad_rounds else
                                      "kavg-async-staleness1" if use_async else "kavg")
        return loss_host / max(num_iterations, 1)

    @torch.no_grad()
    def model_checksum(self) -> float:
        """sum(|x|) over the model's parameters and floating buffers (fp64; one device
        reduction + one read-back).  Reported per task so the job driver can check that
        every active worker holds the same model (elastic resize, K-AVG)."""
        sp = self._flat
        if sp is not None and getattr(sp, "state", None) is not None:
            return float(sp.state[:sp.i64_off].double().abs().sum())
        tot = torch.zeros((), dtype=torch.float64)
        for t in list(self._network.parameters()) + [b for b in self._network.buffers() if b.is_floating_point()]:
            tot += t.detach().double().abs().sum().cpu()
        return float(tot)

    def _sync_optimizer_state(self, comm):
        """Before ragged-tail local rounds of a persistent-state job: a sharded update (engine/dp.py
        shard plan) kept the optimizer state current only on each rank's own chunk; every rank
        zeroes the rest and one SUM all-reduce per state buffer gives all ranks the owners'
        values (a no-op collective when the state is already replicated)."""
        sh = self._shards.get(id(comm))
        if sh is None or sh.region is None or self._flat is None or not hasattr(self.optimizer, "_bufs"):
            return
        names = list(getattr(self.optimizer, "_STATE_NAMES", ()) or ())
        if not names:
            return
        bufs = self.optimizer._bufs(self._flat, names)
        owned = sh.owned()
        for name in names:
            t = bufs[name]
            keep = torch.zeros_like(t)
            for lo, hi in owned:
                keep[lo:hi].copy_(t[lo:hi])
            t.copy_(keep)
            comm.all_reduce_(t)

    def _allreduce_grads_eager(self):
        """Eager (CPU / no-graph) gradient average over the grad-sync group."""
        comm = self._grad_comm
        if self._flat is not None:
            self._flat.finish_grads()
            comm.all_reduce_(self._flat.grad)
            self._flat.grad.div_(comm.world)
            return
        ps = [p for p in self._network.parameters() if p.grad is not None]
        flat = torch.cat([p.grad.reshape(-1) for p in ps])
        comm.all_reduce_(flat)
        flat.div_(comm.world)
        off = 0
        for p in ps:
            p.grad.copy_(flat[off:off + p.numel()].view_as(p.grad))
            off += p.numel()

    def _prime_grad_sync(self):
        """Every rank, same point: one eager all-reduce on the gradient buffer so RCCL's
        connections exist before any graph containing collectives is captured."""
        comm = self._grad_comm
        if self._flat is not None and comm is not None and self.device.type == "cuda":
            comm.all_reduce_(self._flat.grad)

    # ---- job-initialisation warm-up (runs before the job's clock, like init) -----------------
    def _warm(self) -> int:
        """Capture, before the first epoch, the hipGraphs the job's epochs will replay: the
        train step for every minibatch shape of this worker's first epoch, and the eval
        forward for every validation batch shape.  The epoch's batches are planned exactly as
        ``_train`` / ``_validate`` plan them (the resident split uploads the worker's shard to
        HBM here, during initialisation), and each NEW batch shape runs the user's ``train`` /
        ``validate`` once in *dry* mode: ``step`` / ``evaluate`` build and capture their graph
        (capture never mutates training state: engine/step.py) but replay nothing, so the
        model, the optimizer and the BN statistics are untouched.  The reference has no graphs
        to build; its clock (ml/pkg/train/job.go:183) also starts after initialisation.

        A ``train`` written as the reference's manual loop (``loss.backward();
        self.optimizer.step()``, e.g. examples/function_lenet.py) does not go through ``step``,
        so its dry call WOULD update the model: every tensor a training step mutates (flat
        master / shadow / gradients / buffers and counters, or the loose parameters and buffers,
        and the optimizer's state) is snapshotted before the warm-up and restored after it, and
        a dry ``train`` that never called ``step`` ends the train-shape scan (it has no graph to
        capture).  Epoch 1 therefore starts from exactly the recovery-base model.
        Returns the number of graphs captured."""
        self._on_train_start()
        if self.device is None or self.device.type != "cuda" or os.environ.get("KUBEML_NO_GRAPH") == "1":
            return 0
        comm = self._comm()
        N, fid, K = self.args._N, self.args._func_id, self.args._K
        bs = self.batch_size
        splits = split_minibatches(range(self._dataset.num_docs), N)
        assigned = splits[fid]
        per = max(get_subset_period(K, bs, assigned), 1)
        intervals = [(i, min(assigned.stop, i + per)) for i in range(assigned.start, assigned.stop, per)]
        # as in _train: rounds below full_rounds sync gradients, a ragged tail runs local
        full_rounds = min(-(-len(sp) // max(get_subset_period(K, bs, sp), 1)) for sp in splits)
        grad_ok = self._grad_sync_ok(comm, K)
        if grad_ok:
            self._grad_comm = comm
            self._prime_grad_sync()
        done = 0
        snap = self._training_snapshot()
        self._dry = True
        try:
            self._sync_mode = "grad" if grad_ok else "local"
            seen = set()
            manual = False
            streamed = self._dataset._plan_stream("train", intervals, bs, self.device)
            # a resident / streamed split yields batches as device views (cheap to walk); a host
            # loader only walks the first and the last interval (the shapes a ragged end adds)
            rs = range(len(intervals)) if streamed else sorted({0, len(intervals) - 1}) if intervals else []
            for r in rs:
                if manual:
                    break
                i, e = intervals[r]
                self._sync_mode = "grad" if (grad_ok and r < full_rounds) else "local"
                self._dataset._load_train_data(start=i, end=e)
                for batch in self._batches():
                    shape = tuple(getattr(batch[0], "shape", ())) if isinstance(batch, (tuple, list)) else None
                    if (shape, self._sync_mode) in seen:
                        continue
                    seen.add((shape, self._sync_mode))
                    before = self._dry_calls
                    self.train(self._batch_to_device(batch), 0)
                    if self._dry_calls == before:   # a manual loop: it stepped for real (restored below)
                        manual = True
                        break
                    done += 1
            self._dataset._stream_end()
            self._sync_mode = "local"
            if self._dataset.num_val_docs:
                va = split_minibatches(range(self._dataset.num_val_docs), N)[fid]
                seen = set()
                self._network.eval()
                with torch.no_grad():
                    self._dataset._plan_stream("test", [(va.start, va.stop)], bs, self.device)
                    self._dataset._load_validation_data(start=va.start, end=va.stop)
                    for batch in self._batches():
                        shape = tuple(getattr(batch[0], "shape", ())) if isinstance(batch, (tuple, list)) else None
                        if shape in seen:
                            continue
                        seen.add(shape)
                        before = self._dry_calls
                        self.validate(self._batch_to_device(batch), 0)
                        if self._dry_calls == before:   # no evaluate(): nothing to capture
                            break
                        done += 1
                    self._dataset._stream_end()
                self._network.train()
        finally:
            self._dry = False
            self._sync_mode = "local"
            self._grad_comm = None
            self._training_restore(snap)
        torch.cuda.synchronize(self.device)
        return done

    def _training_snapshot(self):
        """(tensors, copies, optimizer host state) of everything a real training step mutates:
        the flat space's state (fp32 master, parameter buffers, i64 counters), gradient and bf16
        shadow — or the loose parameters, gradients and buffers — and the optimizer's device
        state (momenta / moments, step and first-step flags) with its host-side counters."""
        import copy
        ts = []
        sp = self._flat
        if sp is not None and getattr(sp, "state", None) is not None:
            ts += [t for t in (sp.state, sp.grad, getattr(sp, "shadow", None)) if t is not None]
        else:
            ts += [p for p in self._network.parameters()]
            ts += [p.grad for p in self._network.parameters() if p.grad is not None]
            ts += [b for b in self._network.buffers()]
        opt = self.optimizer
        host = None
        if opt is not None:
            if hasattr(opt, "state_tensors"):
                ts += opt.state_tensors()
                # keys are the parameters themselves: copy the values, never the keys
                st = {k: ({n: (v.detach().clone() if torch.is_tensor(v) else copy.copy(v)) for n, v in d.items()}
                          if isinstance(d, dict) else d) for k, d in opt.state.items()}
                host = (st, getattr(opt, "_first", None), getattr(opt, "_step_host", None))
            else:
                host = copy.deepcopy(opt.state_dict())
        seen, uniq = set(), []
        for t in ts:
            if id(t) not in seen:
                seen.add(id(t))
                uniq.append(t)
        with torch.no_grad():
            return uniq, [t.detach().clone() for t in uniq], host

    def _training_restore(self, snap):
        ts, copies, host = snap
        with torch.no_grad():
            for t, c in zip(ts, copies):
                t.copy_(c)
        opt = self.optimizer
        if opt is None or host is None:
            return
        if hasattr(opt, "state_tensors"):
            opt.state.clear()
            opt.state.update(host[0])
            if host[1] is not None:
                opt._first = host[1]
            if host[2] is not None:
                opt._step_host = host[2]
        else:
            opt.load_state_dict(host)

    # ---- validation (network.py:320-360) --------------------------------------------------
    def _on_validation_start(self):
        self._set_device()
        self._network.eval()

    def _validate(self) -> Tuple[float, float, int]:
        self._on_validation_start()
        comm = self._comm()
        assigned = split_minibatches(range(self._dataset.num_val_docs), self.args._N)[self.args._func_id]
        self._dataset._plan_stream("test", [(assigned.start, assigned.stop)], self.batch_size, self.device)
        self._dataset._load_validation_data(start=assigned.start, end=assigned.stop)
        self._averager.broadcast_(comm, 0)
        acc, loss, nb = 0.0, 0.0, 0
        dev_sums = None          # device-side [acc, loss] accumulation (one read-back)
        with torch.no_grad():
            for idx, batch in enumerate(self._batches()):
                _progress()
                batch = self._batch_to_device(batch)
                a, l = self.validate(batch, idx)
                if isinstance(a, torch.Tensor) and isinstance(l, torch.Tensor):
                    v = torch.stack([a.detach().reshape(()).double(), l.detach().reshape(()).double()])
                    dev_sums = v if dev_sums is None else dev_sums.add_(v)
                else:
                    acc += float(a)
                    loss += float(l)
                nb += 1
        if dev_sums is not None:
            a, l = dev_sums.tolist()
            acc += a
            loss += l
        self._network.train()
        self._dataset._stream_end()
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
    MAX_GRAPHS = 8
    PEER_CHECK_EVERY = 16   # verify the peer data plane's checksums every N grad-sync steps
    COMM_TIMING = 50        # sample the in-graph all-reduce every N steps

    def step(self, x, y, loss_fn=None, forward=None):
        """forward + loss + backward + optimizer step for one batch; on the GPU the first
        call for a given batch shape captures a hipGraph (engine/dp.py) that later calls
        replay.  In a K=1 grad-sync round the gradients are all-reduced over the worker
        group inside the step.  Returns the (device) loss tensor.  forward: optional
        ``forward(network, x, y) -> loss`` replacing ``loss_fn(network(x), y)`` — e.g. on-device
        batch preparation (masking) followed by a model call with extra arguments; it is part
        of the captured graph, so it must be a function of x, y and device state only."""
        from ..nn import backward_loss, cross_entropy
        loss_fn = loss_fn or cross_entropy
        if self.device is None or self.device.type != "cuda" or os.environ.get("KUBEML_NO_GRAPH") == "1":
            self.optimizer.zero_grad()
            loss = forward(self._network, x, y) if forward is not None else loss_fn(self(x), y)
            loss.backward()
            if self._sync_mode == "grad":
                self._allreduce_grads_eager()
                self._synced_steps += 1
            self.optimizer.step()
            return loss
        grad = self._sync_mode == "grad"
        comm = self._grad_comm if grad else None
        key = (tuple(x.shape), tuple(y.shape), x.dtype, y.dtype, id(forward or loss_fn), grad,
               id(comm) if comm is not None else None)
        g = self._graphs.get(key)
        if g is None:
            g = self._build_step(key, x, y, loss_fn, comm, forward)
        if self._dry:                 # job warm-up: graph built and captured, nothing replayed
            self._dry_calls += 1
            return torch.zeros((), dtype=torch.float32, device=x.device)
        g["x"].copy_(x, non_blocking=True)
        g["y"].copy_(y, non_blocking=True)
        loss = g["step"]()
        if grad:
            self._synced_steps += 1
        return loss

    def _build_step(self, key, x, y, loss_fn, comm, forward=None):
        """Build and capture the train-step graph for one batch shape (+ comm group)."""
        with trace.span("step_graph", shape=str(tuple(x.shape)), comm=comm.world if comm is not None else 1):
            from ..engine.dp import make_train_step
            if len(self._graphs) >= self.MAX_GRAPHS:
                self._graphs.pop(next(iter(self._graphs)))
            xs, ys = x.clone(), y.clone()
            plan = peer = None
            if comm is not None:
                from ..parallel.plan import choose_plan
                plan = choose_plan(comm.world, self._flat.grad.numel() * 4)
                peer = self._reusable_peer(comm, plan)
            st = make_train_step(self._network, self._flat, self.optimizer, loss_fn, xs, ys,
                                 group=comm.group if comm is not None else None,
                                 world=comm.world if comm is not None else 1,
                                 plan=plan, peer=peer, comm_timing=self.COMM_TIMING if comm is not None else 0,
                                 forward=forward)
            self.logger.info("train step graph: batch %s, comm %s, plan %s, transport %s", tuple(x.shape),
                             comm.world if comm is not None else 1, plan.tag() if plan is not None else None,
                             type(st.peer).__name__ if st.peer is not None else None)
            if st.peer is not None and comm is not None:
                if st.schedule in ("shard", "shardov"):
                    old = self._shards.get(id(comm))
                    if old is not None and old is not st.peer:
                        old.close()                        # collective: every rank builds the same plans
                    self._shards[id(comm)] = st.peer       # bound to this model's flat buffers
                else:
                    comm.grad_peer = st.peer          # one gradient transport per group, reused
            from ..runtime.worker import busy
            with busy(), trace.span("capture"):   # capture + warm-up can take seconds
                st.capture()
            g = self._graphs[key] = {"x": xs, "y": ys, "step": st}
            return g

    def _reusable_peer(self, comm, plan):
        """The transport a new train-step graph may reuse: the shard of this model's space on
        ``comm``, or the group's gradient all-reduce if its slots fit this gradient and wire
        (one that does not is closed — collectively: every rank sees the same sizes)."""
        if plan.backend != "peer":
            return None
        if plan.schedule in ("shard", "shardov", "shardride"):   # all run on the PeerShard of this model's space
            sh = self._shards.get(id(comm))
            return sh if sh is not None and sh.region is not None else None
        gp = getattr(comm, "grad_peer", None)
        if gp is None or gp.region is None:
            return None
        if gp.supports(self._flat.grad, "twoshot", plan.wire_dtype):
            return gp
        gp.close()
        comm.grad_peer = None
        return None

    def evaluate(self, x, y, loss_fn=None, forward=None):
        """Eval-mode forward + loss + correct count for one validation batch -> (correct,
        loss) as device tensors.  On the GPU the first call per batch shape captures the
        forward into a hipGraph that later calls replay: a validation pass is then one replay
        per batch instead of ~80 host-issued launches (host-bound at the reference's batch
        sizes).  Weights and BN running statistics are read in place, so every replay sees
        the current model.  forward: optional ``forward(network, x, y) -> (correct, loss)``
        replacing the classifier default (captured like the default)."""
        from ..nn import cross_entropy
        loss_fn = loss_fn or cross_entropy

        def fwd(xx, yy):
            if forward is not None:
                return forward(self._network, xx, yy)
            out = self._network(xx)
            if loss_fn is cross_entropy:
                return loss_fn(out, yy, return_correct=True)[::-1]
            loss = loss_fn(out, yy)
            return (out.argmax(1) == yy).sum(), loss

        if self.device is None or self.device.type != "cuda" or os.environ.get("KUBEML_NO_GRAPH") == "1":
            return fwd(x, y)
        key = ("eval", tuple(x.shape), tuple(y.shape), x.dtype, y.dtype, id(forward or loss_fn))
        g = self._eval_graphs.get(key)
        if g is None:
            if len(self._eval_graphs) >= self.MAX_GRAPHS:
                self._eval_graphs.pop(next(iter(self._eval_graphs)))
            _sp = trace.span("eval_graph", shape=str(tuple(x.shape)))
            _sp.__enter__()
            xs, ys = x.clone(), y.clone()
            s = torch.cuda.Stream(device=self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                fwd(xs, ys)                       # warm-up: plans, workspaces, lazy buffers
            torch.cuda.current_stream(self.device).wait_stream(s)
            graph = torch.cuda.CUDAGraph()
            from ..engine.step import capture_graph
            with capture_graph(graph):
                outs = fwd(xs, ys)
            g = self._eval_graphs[key] = {"x": xs, "y": ys, "graph": graph, "out": outs}
            _sp.__exit__(None, None, None)
        if self._dry:                 # job warm-up: captured, not replayed
            self._dry_calls += 1
            z = torch.zeros((), dtype=torch.float32, device=x.device)
            return z, z.clone()
        g["x"].copy_(x, non_blocking=True)
        g["y"].copy_(y, non_blocking=True)
        g["graph"].replay()
        correct, loss = g["out"]
        return correct.clone(), loss.clone()

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
