"""TrainJob — per-job orchestrator (reference ml/pkg/train/job.go:22-451,
function.go:44-227, util.go:20-280).

Same epoch loop and semantics as the reference:

* ``init`` task on worker 0 → layer names (job.go:268-291);
* per epoch: fan the ``train`` task out to workers ``[0, P)`` with ``N=P``; the K-AVG
  rounds inside the epoch are RCCL all-reduces between the workers themselves (no
  ``/next`` barrier, no merger goroutine); loss = mean over the workers that answered
  (util.go:82-95); partial failure tolerated, total failure fails the job
  (util.go:144-166);
* history: ``train_loss``, ``parallelism``, cumulative ``epoch_duration``
  (util.go:36-50; job.go:321-327), metrics pushed to the PS after every update;
* if not static and not the last epoch: ask the scheduler for the next parallelism
  and wait for the answer (job.go:196-215); ``DEBUG_ENV`` / ``LIMIT_PARALLELISM``
  freeze it (job.go:210);
* validation every ``validate_every`` epochs except the last, then once at the end
  unless the goal accuracy stopped the job (job.go:218-263); sample-weighted
  averages (util.go:100-122);
* force stop via :meth:`stop` (job.go:239-244).

Beyond the reference: a reference-model checkpoint after init and
after every epoch (safetensors, torch ``state_dict`` names); a lost worker makes the
pool rebuild on the surviving GPUs, restore the last checkpoint and re-run the epoch
(bounded retries); history is persisted after every epoch.
"""
from __future__ import annotations

import json
import logging
import os
import queue
import threading
import time
from typing import Callable, Dict, List, Optional

from ..api.errors import KubeMLException
from ..api.types import JobHistory, JobState, History, TrainTask
from ..metrics import latest_metrics
from ..store.ckpt import ckpt_path
from ..utils import trace


class JobLogger:
    """Structured per-job log: ``<store>/logs/<jobId>.log`` (JSON lines), the source of
    ``kubeml logs --id`` (reference wraps ``kubectl logs job-{id}``, cli/log.go:28-65)."""

    def __init__(self, store_dir: str, job_id: str):
        d = os.path.join(store_dir, "logs")
        os.makedirs(d, exist_ok=True)
        self.path = os.path.join(d, f"{job_id}.log")
        self._f = open(self.path, "a", buffering=1)
        self._py = logging.getLogger(f"kubeml.job.{job_id}")
        self._lock = threading.Lock()

    def _w(self, level: str, msg: str, **kw):
        rec = {"ts": time.time(), "level": level, "msg": msg, **kw}
        with self._lock:
            try:
                self._f.write(json.dumps(rec, default=str) + "\n")
            except ValueError:
                pass
        getattr(self._py, level if level != "warn" else "warning")("%s %s", msg, kw if kw else "")

    def info(self, msg, **kw):
        self._w("info", msg, **kw)

    def warn(self, msg, **kw):
        self._w("warn", msg, **kw)

    def error(self, msg, **kw):
        self._w("error", msg, **kw)

    def debug(self, msg, **kw):
        self._w("debug", msg, **kw)

    def close(self):
        with self._lock:
            self._f.close()


class JobError(KubeMLException):
    pass


class TrainJob:
    MAX_RECOVERIES = 3

    def __init__(self, task: TrainTask, *, code_path: str, store_dir: str, pool_factory: Callable,
                 on_metrics: Callable, on_finish: Callable, request_update: Optional[Callable] = None,
                 history_store=None, max_parallelism: int = 8, freeze_parallelism: bool = False,
                 task_timeout: float = 3600.0, inventory=None):
        self.task = task
        self.id = task.job.id
        self.req = task.request
        opts = self.req.options
        self.static = bool(opts.static_parallelism)
        # capture the workers' graphs during initialisation (KUBEML_WARM=0: inside epoch 1)
        self.warm = os.environ.get("KUBEML_WARM", "1") != "0"
        self.validate_every = int(opts.validate_every)
        self.goal_accuracy = float(opts.goal_accuracy)
        self.K = int(opts.k)
        self.sync = str(getattr(opts, "sync", "") or "")
        self.code_path = code_path
        self.store_dir = store_dir
        self.pool_factory = pool_factory
        self.on_metrics = on_metrics
        self.on_finish = on_finish
        self.request_update = request_update
        self.history_store = history_store
        self.freeze = freeze_parallelism
        self.task_timeout = task_timeout
        self.max_parallelism = max(1, int(max_parallelism))
        self.parallelism = self._clamp(task.job.state.parallelism or opts.default_parallelism)
        self.history = JobHistory()
        self.epoch = 0
        self.exit_err: Optional[str] = None
        self.accuracy_reached = False
        self.sched_q: "queue.Queue[JobState]" = queue.Queue()
        self._stop = threading.Event()
        self.pool = None
        self.log = JobLogger(store_dir, self.id)
        self.ckpt = ckpt_path(store_dir, self.id)
        self.have_ckpt = False
        self.ckpt_epoch = None                # epoch of the last checkpoint confirmed on disk
        self.thread: Optional[threading.Thread] = None
        self.images_per_second = 0.0
        self.last_sync_seconds = 0.0
        self.last_grad_rounds = 0
        self.done = threading.Event()
        self.resume_from = getattr(opts, "resume_from", "") or ""
        self.inventory = inventory
        self._shrink_to = None
        self.checksums: List[Dict] = []   # per epoch: {rank: (start, end)} model checksums
        self._pending_restore = None
        self.start_epoch = 1

    # ------------------------------------------------------------------ control
    def start(self) -> "TrainJob":
        self.thread = threading.Thread(target=self.run, name=f"job-{self.id}", daemon=True)
        self.thread.start()
        return self

    def update(self, state: JobState):
        """Scheduler answer (reference POST /update → schedulerCh, train/api.go:69-96)."""
        self.sched_q.put(state)

    def stop(self):
        self._stop.set()

    def router(self):
        """The job's own REST surface (reference ml/pkg/train/api.go:141-149).  ``/next``
        is gone: the K-AVG barrier is the RCCL all-reduce between the workers."""
        from .http import Router
        r = Router(f"job-{self.id}")
        r.add("POST", "/start", lambda q: (self.start() and "") if self.thread is None else "")
        r.add("POST", "/update", lambda q: self.update(JobState.from_dict(q.json())) or "")
        r.add("DELETE", "/stop", lambda q: self.stop() or "")
        r.add("GET", "/health", lambda q: "")
        r.add("GET", "/status", lambda q: {"id": self.id, "epoch": self.epoch, "parallelism": self.parallelism,
                                           "history": self.history.to_dict(), "done": self.done.is_set(),
                                           "error": self.exit_err})
        return r

    def _clamp(self, p) -> int:
        return max(1, min(int(p), self.max_parallelism))

    # ------------------------------------------------------------------ worker fan-out
    def _msg(self, kind: str, **kw) -> Dict:
        m = {"op": "task", "kind": kind, "job": self.id, "function": self.req.function_name,
             "code_path": self.code_path, "N": self.parallelism, "K": self.K, "batch_size": self.req.batch_size,
             "lr": self.req.lr, "epoch": self.epoch}
        if self.sync:
            m["sync"] = self.sync
        m.update(kw)
        return m

    def _ensure_pool(self):
        if self.pool is None or self.pool.broken:
            if self.pool is not None:
                self.pool.shutdown(force=True)
            self.pool = self.pool_factory(self)
            self.max_parallelism = min(self.max_parallelism, self.pool.n)
            self.parallelism = self._clamp(self.parallelism)

    def _maybe_release_idle(self):
        """Epoch boundary: an elastic job holding more slots than its parallelism gives
        the idle ones back when another job is waiting for slots (the pool is rebuilt on
        the kept GPUs and restores the just-written checkpoint)."""
        inv = self.inventory
        if inv is None or self.pool is None or self.pool.broken or not self.have_ckpt:
            return
        if inv.waiting > 0 and self.pool.n > self.parallelism:
            self.log.info("releasing idle workers", keep=self.parallelism, had=self.pool.n)
            self._shrink_to = self.parallelism
            self.pool.broadcast({"op": "release", "job": self.id}, timeout=60)
            self.pool.shutdown()
            self.pool = None
            self.max_parallelism = self.parallelism
            self._pending_restore = self.ckpt

    def _fanout(self, kind: str, ranks: List[int], **kw) -> Dict[int, Dict]:
        msgs = {r: self._msg(kind, **kw) for r in ranks}
        with trace.span(f"fanout:{kind}", epoch=self.epoch, N=len(ranks)):
            return self.pool.run(msgs, timeout=self.task_timeout)

    # ------------------------------------------------------------------ phases
    def _init(self):
        self._ensure_pool()
        rep = self.pool.call(0, self._msg("init", N=1))
        if not rep.get("ok"):
            raise JobError(f"error invoking init function: {rep.get('error')}", rep.get("code", 500))
        layers = rep.get("result") or []
        if len(layers) == 0:
            raise JobError("length of the layers is zero", 500)
        self.log.info("model initialised", layers=len(layers))
        if self.resume_from:
            self._resume()
        else:
            self._checkpoint(wait=True)   # the recovery base: confirmed on disk before epoch 1
        self._warm()
        return layers

    def _warm(self):
        """Part of initialisation (before the clock starts, as init is in job.go:173-183): every
        worker of the first epoch captures the train-step and eval graphs of its batch shapes
        (KubeModel._warm; no update is applied).  Best effort: a failure only costs the
        capture time inside epoch 1."""
        if not self.warm:
            return
        try:
            P = self.parallelism
            res = self._fanout("warm", list(range(P)), N=P, restore=self._pending_restore)
            bad = {r: v.get("error") for r, v in res.items() if not v.get("ok")}
            if bad:
                self.log.warn("warm-up failed on some workers", errors=bad)
            else:
                self.log.info("workers warm", shapes={str(r): v.get("result") for r, v in sorted(res.items())})
        except Exception as e:
            self.log.warn("warm-up skipped", error=repr(e))

    def _resume(self):
        """Continue job ``resume_from``: its checkpoint becomes this job's starting model
        (rank 0 loads it, the epoch-start broadcast spreads it), its history and epoch
        index carry over."""
        import shutil
        src = ckpt_path(self.store_dir, self.resume_from)
        if not os.path.exists(src):
            raise JobError(f"no checkpoint for job {self.resume_from}", 404)
        shutil.copyfile(src, self.ckpt)
        if os.path.exists(src + ".json"):
            shutil.copyfile(src + ".json", self.ckpt + ".json")
            with open(src + ".json") as f:
                meta = json.load(f)
            self.start_epoch = int(meta.get("epoch", 0)) + 1
            if meta.get("history"):
                self.history = JobHistory.from_dict(meta["history"])
        if self.history_store is not None and self.history_store.exists(self.resume_from):
            self.history = self.history_store.get(self.resume_from).data
        self.have_ckpt = True
        self._pending_restore = self.ckpt
        self.log.info("resuming", source=self.resume_from, start_epoch=self.start_epoch)

    def _checkpoint(self, wait: bool = False):
        """Rank 0 snapshots the reference model and writes it in the background (off the
        epoch's critical path); ``wait`` = the file is on disk when this returns."""
        rep = self.pool.call(0, {"op": "checkpoint", "job": self.id, "path": self.ckpt, "epoch": self.epoch,
                                 "extra": {"history": self.history.to_dict()}, "wait": bool(wait)})
        if rep.get("previous_error"):
            self.log.warn("background checkpoint write failed", error=rep["previous_error"],
                          durable_epoch=rep.get("durable_epoch"))
        if not rep.get("ok"):
            self.log.warn("checkpoint failed", error=rep.get("error"))
        # have_ckpt = some checkpoint is CONFIRMED on disk (a waited write, or an earlier
        # background write that completed); a restore then reads the last good file
        if rep.get("durable_epoch") is not None:
            self.have_ckpt = True
        self.ckpt_epoch = rep.get("durable_epoch")

    def _train_epoch(self) -> float:
        """One epoch with recovery: a lost worker → rebuild the pool on the survivors,
        restore the last checkpoint and re-run the epoch."""
        for attempt in range(self.MAX_RECOVERIES + 1):
            self._ensure_pool()
            P = self.parallelism
            restore = self.ckpt if (attempt > 0 and self.have_ckpt) else self._pending_restore
            t0 = time.time()
            res = self._fanout("train", list(range(P)), N=P, restore=restore)
            ok = {r: v for r, v in res.items() if v.get("ok")}
            bad = {r: v for r, v in res.items() if not v.get("ok")}
            if not bad:
                self._pending_restore = None
                losses = [float(v["result"]["loss"]) for v in ok.values()]
                self.checksums.append({r: (v.get("start_checksum"), v.get("end_checksum")) for r, v in ok.items()})
                hbm = max((v.get("hbm_bytes", 0) for v in ok.values()), default=0)
                self.last_sync_seconds = max((v.get("sync_seconds", 0.0) for v in ok.values()), default=0.0)
                self.last_grad_rounds = max((v.get("grad_rounds", 0) for v in ok.values()), default=0)
                modes = sorted({v.get("sync_mode") for v in ok.values() if v.get("sync_mode")})
                if modes:
                    self.history.sync_mode.append("+".join(modes))
                self._epoch_stats(time.time() - t0, hbm)
                return sum(losses) / len(losses)
            errs = "; ".join(f"worker {r}: {v.get('error')}" for r, v in sorted(bad.items()))
            dead = [r for r, v in bad.items() if v.get("dead") or v.get("hung")]   # hung = lost
            self.log.warn("epoch failed", epoch=self.epoch, attempt=attempt, errors=errs, dead=dead)
            if not dead and self.pool is not None and not self.pool.broken:
                # function error on a healthy pool (no lost peer): the reference fails the
                # epoch only if every function failed, but with collectives a partial
                # result is an incomplete average, so the error is reported as-is
                raise JobError(f"all functions finished with an error: {errs}", 500)
            if not self.have_ckpt:
                raise JobError(f"worker lost before the first checkpoint: {errs}", 500)
            survivors = max(1, (self.pool.n if self.pool else 1) - len(dead))
            self.max_parallelism = min(self.max_parallelism, survivors)
            self.parallelism = self._clamp(min(self.parallelism, survivors))
            self.pool.shutdown(force=True)
            self.pool = None
            self._shrink_to = survivors
            self.log.warn("recovering", survivors=survivors, parallelism=self.parallelism)
        raise JobError(f"epoch {self.epoch} failed after {self.MAX_RECOVERIES} recoveries", 500)

    def _epoch_stats(self, seconds: float, hbm: int):
        self.last_epoch_seconds = seconds
        self.last_hbm = hbm

    def _validate(self):
        """Sample-weighted validation over the active workers (util.go:100-122)."""
        self._ensure_pool()
        P = self.parallelism
        res = self._fanout("val", list(range(P)), N=P)
        acc = loss = total = 0.0
        n_ok = 0
        for r, v in sorted(res.items()):
            if not v.get("ok"):
                self.log.warn("validation function failed", worker=r, error=v.get("error"))
                continue
            d = v["result"]
            ln = float(d.get("length", 0))
            acc += float(d["accuracy"]) * ln
            loss += float(d["loss"]) * ln
            total += ln
            n_ok += 1
        if n_ok == 0:
            raise JobError("all validation functions failed", 500)
        if total > 0:
            acc /= total
            loss /= total
        self.history.validation_loss.append(loss)
        self.history.accuracy.append(acc)
        self._push_metrics()
        self.log.info("validation", epoch=self.epoch, accuracy=acc, loss=loss, samples=total)
        if acc >= self.goal_accuracy:
            self.log.info("goal accuracy reached", goal=self.goal_accuracy, accuracy=acc)
            self.accuracy_reached = True

    def _push_metrics(self):
        try:
            self.on_metrics(self.id, latest_metrics(self.history), self)
        except Exception as e:  # reference logs and continues (job.go:300-303)
            self.log.warn("error updating metrics", error=repr(e))

    def _save_history(self):
        if self.history_store is None:
            return
        self.history_store.save(History(id=self.id, task=self.req, data=self.history))

    def _next_parallelism(self):
        """Scheduler round-trip (job.go:196-215)."""
        if self.request_update is None:
            return
        self.task.job.state.parallelism = self.parallelism
        try:
            self.request_update(self.task)
        except Exception as e:
            self.log.error("error updating parallelism", error=repr(e))
            return
        try:
            st = self.sched_q.get(timeout=60)
        except queue.Empty:
            self.log.warn("no answer from the scheduler; keeping parallelism")
            return
        self.task.job.state = st
        if not self.freeze:
            self.parallelism = self._clamp(st.parallelism)
        self.log.info("next config from the scheduler", parallelism=self.parallelism)

    # ------------------------------------------------------------------ main loop
    def run(self):
        self.log.info("starting train job", request=self.req.to_dict())
        try:
            self._init()
            prior = self.history.epoch_duration[-1] if (self.resume_from and self.history.epoch_duration) else 0.0
            start = time.time() - prior  # epoch_duration stays cumulative across a resume
            E = int(self.req.epochs)
            for self.epoch in range(self.start_epoch, E + 1):
                t0 = time.time()
                with trace.span("epoch", epoch=self.epoch, P=self.parallelism):
                    loss = self._train_epoch()
                elapsed = time.time() - t0
                self.task.job.state.elapsed_time = elapsed
                n_imgs = self._epoch_samples()
                self.images_per_second = n_imgs / max(elapsed, 1e-9) if n_imgs else 0.0
                self.history.parallelism.append(float(self.parallelism))
                self.history.epoch_duration.append(time.time() - start)  # cumulative (job.go:327)
                self.history.train_loss.append(loss)
                self._push_metrics()
                self.log.info("epoch finished", epoch=self.epoch, loss=loss, seconds=elapsed,
                              parallelism=self.parallelism, images_per_second=self.images_per_second,
                              sync_seconds=self.last_sync_seconds, grad_sync_rounds=self.last_grad_rounds,
                              checksums={str(r): c for r, c in sorted(self.checksums[-1].items())}
                              if self.checksums else None)
                if not self.static and self.epoch < E:
                    self._next_parallelism()
                if self.validate_every and self.epoch % self.validate_every == 0 and self.epoch != E:
                    try:
                        self._validate()
                    except Exception as e:
                        self.log.error("error performing validation", error=repr(e))
                self._checkpoint()
                self._save_history()
                self._maybe_release_idle()
                if self._stop.is_set():
                    self.accuracy_reached = True
                    self.exit_err = "job was force stopped"
                    break
                if self.accuracy_reached:
                    break
            if not self.accuracy_reached and self.epoch >= self.start_epoch:
                try:
                    self._validate()
                except Exception as e:
                    self.log.error("error performing validation", error=repr(e))
            self._checkpoint(wait=True)          # inference / resume read it right after
            self._save_history()
            self.log.info("training finished", epochs=self.epoch, history=self.history.to_dict())
        except Exception as e:
            self.exit_err = getattr(e, "message", None) or repr(e)
            self.log.error("job failed", error=self.exit_err)
            try:
                self._save_history()
            except Exception:
                pass
        finally:
            if self.pool is not None:
                try:
                    if not self.pool.broken:
                        self.pool.broadcast({"op": "release", "job": self.id}, timeout=60)
                finally:
                    self.pool.shutdown()
                    self.pool = None
            if trace.enabled():
                trace.flush(os.path.join(self.store_dir, "traces"))
            self.done.set()
            try:
                self.on_finish(self.id, self.exit_err)
            finally:
                self.log.close()

    def _epoch_samples(self) -> int:
        try:
            from ..store.shards import ShardStore
            from ..api.types import STORAGE_SUBSET_SIZE
            m = ShardStore(self.store_dir).manifest(self.req.dataset)
            return int(m["train"]["n"])
        except Exception:
            return 0
