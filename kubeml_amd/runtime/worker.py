"""Resident worker process — one per MI355X (replaces the Fission function pods).

Reference: every train/val/init/infer call is an HTTP GET to a Fission function pod
running a Flask app that imports the user's file and calls ``main()``
(ml/environment/server.py:60-128); state moves through RedisAI between calls
(python/kubeml/kubeml/network.py:424-461).

MI355X-native: a worker is a long-lived process bound to ONE GPU (``GPU_ID`` →
``torch.cuda.set_device``) and a member of the job's ``torch.distributed`` world
(``nccl`` = RCCL over xGMI on GPUs, ``gloo`` on CPU) with pre-built sub-groups for
every parallelism ``p`` (elastic resize = pick the sub-communicator of ranks
``[0, p)``).  It receives task descriptors over a pipe from the job
driver, runs them in a :class:`TaskContext`, and keeps the job's ``KubeModel`` (network,
optimizer, flat parameter buffers, graphs) resident in HBM between tasks: the user's
``main()`` runs once per job; later tasks call ``start()`` on the cached model.

Messages (dicts): ``{"op": "task", "kind": init|train|val|infer, ...}``,
``{"op": "checkpoint", "job", "path", "epoch"}``, ``{"op": "release", "job"}``,
``{"op": "stats"}``, ``{"op": "shutdown"}``.  Replies: ``{"ok": True, "result": ...}`` or
the error envelope ``{"ok": False, "error", "code"}`` (server.py:133-151).
"""
from __future__ import annotations

import importlib.util
import logging
import os
import sys
import time
import traceback
from datetime import timedelta
from typing import Any, Dict

log = logging.getLogger("kubeml.worker")

_PROGRESS = None   # (shared array, rank): bumped by progress(); watched by the pool


def _jsonable(x):
    import numpy as np
    try:
        import torch
        if isinstance(x, torch.Tensor):
            return x.detach().cpu().tolist()
    except Exception:
        pass
    if isinstance(x, np.ndarray):
        return x.tolist()
    if isinstance(x, (np.floating, np.integer)):
        return x.item()
    if isinstance(x, dict):
        return {str(k): _jsonable(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_jsonable(v) for v in x]
    return x


def progress(n: int = 1):
    """Mark forward progress of this worker (a K-AVG round, a minibatch).  The pool
    declares a rank hung when its counter stops while its peers' advance."""
    if _PROGRESS is not None:
        arr, rank = _PROGRESS
        arr[rank] += n


class busy:
    """Keep this worker's progress counter moving during a long phase that makes no
    K-AVG / minibatch progress of its own (first native build, checkpoint restore, graph
    capture, importing the user's file): a heartbeat thread ticks every ``interval`` seconds,
    so the pool's stall watchdog only fires on a real hang.  No-op outside a pool worker."""

    def __init__(self, interval: float = 5.0):
        self.interval = interval
        self._stop = None
        self._t = None

    def __enter__(self):
        if _PROGRESS is None:
            return self
        import threading
        self._stop = threading.Event()

        def tick():
            while not self._stop.wait(self.interval):
                progress()
        progress()
        self._t = threading.Thread(target=tick, name="kubeml-busy", daemon=True)
        self._t.start()
        return self

    def __exit__(self, *exc):
        if self._stop is not None:
            self._stop.set()
            self._t.join()
            progress()
        return False


def load_function(path: str, name: str):
    """Import the user's function file under a unique module name (``/specialize``)."""
    mod_name = f"kubeml_fn_{name}_{abs(hash((path, os.path.getmtime(path)))) % 10**8}"
    mod = sys.modules.get(mod_name)
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(mod_name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[mod_name] = mod
    with busy():
        spec.loader.exec_module(mod)
    if not hasattr(mod, "main"):
        raise AttributeError(f"function {name} has no main()")
    return mod


class Worker:
    def __init__(self, rank: int, world: int, opts: Dict[str, Any]):
        self.rank, self.world, self.opts = rank, world, opts
        self.use_gpu = bool(opts.get("use_gpu"))
        self.store_dir = opts["store_dir"]
        self.jobs: Dict[str, Any] = {}       # job id -> KubeModel (resident)
        self.job_fn: Dict[str, str] = {}     # job id -> function code path
        self.device = None
        self.comm = None
        self.store = None
        self.ckpt = None                     # AsyncCheckpointer (background writes)

    # ------------------------------------------------------------------ setup
    def setup(self):
        import torch
        from ..parallel.comm import LocalComm, TorchComm
        from ..store.shards import ShardStore
        from ..utils import trace
        trace.set_process("worker", self.rank)
        gpu_ids = self.opts.get("gpu_ids") or []
        if self.use_gpu:
            gid = int(gpu_ids[self.rank]) if gpu_ids else self.rank
            os.environ["GPU_ID"] = str(gid)
            torch.cuda.set_device(gid)
            self.device = torch.device("cuda", gid)
        else:
            self.device = torch.device("cpu")
            torch.set_num_threads(max(1, int(self.opts.get("threads", 1))))
        if self.world > 1:
            import torch.distributed as dist
            mode = self.opts.get("comm") or ("nccl" if self.use_gpu else "gloo")
            if mode not in ("nccl", "gloo", "gloo+peer"):
                raise ValueError(f"worker comm mode {mode!r}: nccl | gloo | gloo+peer")
            kw = {}
            if mode == "nccl":
                kw["device_id"] = self.device
            dist.init_process_group("nccl" if mode == "nccl" else "gloo",
                                    init_method=f"tcp://127.0.0.1:{self.opts['port']}", rank=self.rank,
                                    world_size=self.world, timeout=timedelta(seconds=self.opts.get("timeout", 600)),
                                    **kw)
            self.comm = TorchComm(peer_data=(mode == "gloo+peer" and self.use_gpu))
            self.comm.prepare_subgroups(self.world)
            if self.use_gpu and os.environ.get("KUBEML_PEER", "0") == "1":
                # fp32 reductions over the world group (K-AVG rounds, BN statistics, counts) go
                # through the peer-memory all-reduce over xGMI instead of RCCL
                self.comm.enable_peer()
        else:
            self.comm = LocalComm()
        self.store = ShardStore(self.store_dir)
        # a resident worker starts warm (the reference's Fission pool keeps pre-specialised
        # containers): the first ``torch.optim`` construction of a user function imports
        # torch._dynamo, ~1.4 s that would otherwise land inside the job's first epoch
        with busy():
            import torch._dynamo  # noqa: F401

    # ------------------------------------------------------------------ ops
    def handle(self, msg: Dict[str, Any]) -> Dict[str, Any]:
        op = msg.get("op")
        if op == "task":
            return self._task(msg)
        if op == "checkpoint":
            return self._checkpoint(msg)
        if op == "release":
            self._release(msg.get("job"))
            return {"ok": True, "result": None}
        if op == "stats":
            return {"ok": True, "result": self._stats()}
        return {"ok": False, "error": f"unknown op {op!r}", "code": 400}

    def _task(self, msg):
        from ..api.errors import KubeMLException
        from ..sdk.context import TaskContext, reset_task, set_task
        from ..utils import fault, trace
        kind = msg["kind"]
        job = msg["job"]
        P = int(msg.get("N", 1))
        ctx = TaskContext(job_id=job, N=P, K=int(msg.get("K", -1)), task=kind, func_id=self.rank,
                          lr=float(msg.get("lr", 0.01)), batch_size=int(msg.get("batch_size", 64)),
                          epoch=int(msg.get("epoch", 1)), data=msg.get("data"),
                          comm=self.comm.sub(P) if P > 1 else _local(), store=self.store,
                          store_dir=self.store_dir, device=self.device, checkpoint=msg.get("checkpoint"))
        ctx.extra["restore"] = msg.get("restore")
        ctx.extra["sync"] = msg.get("sync", "")
        if msg.get("restore") or kind == "infer":
            self._flush_checkpoint()         # the file a restore / inference reads is complete
        token = set_task(ctx)
        t0 = time.perf_counter()
        try:
            fault.point("task", rank=self.rank, epoch=ctx.epoch, task=kind, job=job)
            progress()
            with trace.span(f"task:{kind}", job=job, epoch=ctx.epoch, N=P):
                km = self.jobs.get(job)
                if km is not None and self.job_fn.get(job) == msg["code_path"]:
                    res = km.start()
                else:
                    mod = load_function(msg["code_path"], msg.get("function", "fn"))
                    res = mod.main()
                    km = ctx.extra.get("kubemodel")
                    if km is not None:
                        self.jobs[job] = km
                        self.job_fn[job] = msg["code_path"]
            if self.comm is not None:
                self.comm.check()       # a timed-out peer collective fails the task, loudly
            out = {"ok": True, "result": _jsonable(res), "seconds": time.perf_counter() - t0,
                   "sync_seconds": float(ctx.extra.get("sync_seconds", 0.0)),
                   "start_checksum": ctx.extra.get("start_checksum"),
                   "end_checksum": ctx.extra.get("end_checksum"),
                   "grad_rounds": int(ctx.extra.get("grad_rounds", 0)),
                   "sync_mode": ctx.extra.get("sync_mode")}
            if self.use_gpu:
                import torch
                out["hbm_bytes"] = int(torch.cuda.max_memory_allocated(self.device))
            return out
        except KubeMLException as e:
            return {"ok": False, **e.to_dict()}
        except Exception as e:
            return {"ok": False, "error": repr(e), "code": 500, "traceback": traceback.format_exc()}
        finally:
            reset_task(token)
            if trace.enabled():
                trace.flush(os.path.join(self.store_dir, "traces"))

    def _checkpoint(self, msg):
        """Snapshot now, write in the background (``"wait": True`` — job end, before a
        restore — returns only once the file is on disk)."""
        from ..store.ckpt import AsyncCheckpointer
        km = self.jobs.get(msg["job"])
        if km is None:
            return {"ok": False, "error": f"job {msg['job']} has no model on worker {self.rank}", "code": 404}
        if self.ckpt is None:
            self.ckpt = AsyncCheckpointer()
        try:
            prev = self.ckpt.save(km.network, msg["path"], job_id=msg["job"], epoch=int(msg.get("epoch", 0)),
                                  extra=msg.get("extra"))
            if msg.get("wait"):
                self.ckpt.wait()
        except Exception as e:
            return {"ok": False, "error": f"checkpoint failed: {e!r}", "code": 500,
                    "durable_epoch": self.ckpt.durable_epoch}
        rep = {"ok": True, "result": msg["path"], "durable_epoch": self.ckpt.durable_epoch}
        if prev is not None:
            rep["previous_error"] = repr(prev)
        return rep

    def _flush_checkpoint(self):
        """Wait for the background write.  A failed write is not fatal here: the file
        on disk is still the last good checkpoint (writes rename into place)."""
        if self.ckpt is not None:
            e = self.ckpt.wait(raise_error=False)
            if e is not None:
                log.warning("checkpoint write failed (%r); the checkpoint of epoch %s stays current",
                            e, self.ckpt.durable_epoch)

    def _release(self, job):
        self._flush_checkpoint()
        self.jobs.pop(job, None)
        self.job_fn.pop(job, None)
        import gc
        gc.collect()
        if self.use_gpu:
            import torch
            torch.cuda.empty_cache()

    def _stats(self):
        s = {"rank": self.rank, "world": self.world, "jobs": list(self.jobs), "device": str(self.device)}
        if self.use_gpu:
            import torch
            s["hbm_allocated"] = int(torch.cuda.memory_allocated(self.device))
            s["hbm_reserved"] = int(torch.cuda.memory_reserved(self.device))
        return s

    def shutdown(self):
        try:
            import torch.distributed as dist
            if dist.is_initialized():
                dist.destroy_process_group()
        except Exception:
            pass


def _local():
    from ..parallel.comm import LocalComm
    return LocalComm()


def worker_entry(rank: int, world: int, conn, opts: Dict[str, Any], progress_arr=None):
    """Process entry point (multiprocessing spawn target)."""
    global _PROGRESS
    if progress_arr is not None:
        _PROGRESS = (progress_arr, rank)
    for k, v in (opts.get("env") or {}).items():
        os.environ[k] = str(v)
    logging.basicConfig(level=os.environ.get("KUBEML_LOG_LEVEL", "WARNING"),
                        format=f"%(asctime)s worker{rank} %(name)s %(levelname)s %(message)s")
    w = Worker(rank, world, opts)
    try:
        w.setup()
    except Exception as e:
        conn.send({"ok": False, "error": f"worker {rank} setup failed: {e!r}", "code": 500,
                   "traceback": traceback.format_exc()})
        return
    conn.send({"ok": True, "result": "ready", "rank": rank})
    while True:
        try:
            msg = conn.recv()
        except (EOFError, OSError):
            break
        if msg.get("op") == "shutdown":
            conn.send({"ok": True, "result": "bye"})
            break
        conn.send(w.handle(msg))
    w.shutdown()
