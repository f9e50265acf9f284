"""Parameter server = job manager + GPU inventory + metrics (reference
ml/pkg/ps/{parameter_server.go, api.go, job_pod.go, metrics.go}).

The reference PS creates a k8s pod+service per job (job_pod.go) and relays scheduler
updates, metrics and finish notifications; the model averaging it is named after
happens in the job's RedisAI merger.  Here the PS:

* owns the node's worker slots (one per MI355X; CPU slots when no GPU) and hands each
  job a set of them — jobs run concurrently on disjoint GPUs; a static job takes exactly
  its parallelism, an elastic job up to ``max_parallelism`` and returns idle slots at an
  epoch boundary when another job is waiting; a job waits while too few are free;
* starts a :class:`TrainJob` thread per task (``POST /start``) whose worker pool is
  spawned on the job's GPUs (``runtime.pool``);
* relays ``POST /update/{id}`` (JobState) to the job, keeps Prometheus gauges from
  ``POST /metrics/{id}`` (served on ``:8080/metrics``), ``POST /finish/{id}`` clears
  them and tells the scheduler (api.go:266-327), ``DELETE /stop/{id}`` force-stops,
  ``GET /tasks`` lists running tasks;
* serves inference on a resident 1-worker pool against the job's checkpoint.
"""
from __future__ import annotations

import logging
import os
import threading
import time
from typing import Dict, List, Optional

from ..api.errors import BadRequestError, KubeMLException, NotFoundError
from ..api.types import InferRequest, JobState, MetricUpdate, TrainTask
from ..metrics import Metrics
from ..runtime.pool import WorkerPool
from ..store.ckpt import ckpt_path
from ..store.functions import FunctionStore
from ..store.history import HistoryStore
from .http import Router
from .job import TrainJob

log = logging.getLogger("kubeml.ps")


class Inventory:
    """Worker slots of this node (GPU indices, or CPU slots).

    ``acquire(want, at_least)`` blocks until ``at_least`` slots are free, then takes up
    to ``want`` of them; ``waiting`` counts blocked acquirers so elastic jobs can hand
    idle slots back when another job needs them."""

    def __init__(self, n: int, use_gpu: bool):
        self.n = n
        self.use_gpu = use_gpu
        self.free = list(range(n))
        self.cv = threading.Condition()
        self.waiting = 0
        self.reclaimers = []      # callables that free idle slots (e.g. the inference pool)

    def acquire(self, want: int, stop: Optional[threading.Event] = None, timeout: float = 86400,
                at_least: int = 1) -> List[int]:
        want = max(1, min(want, self.n))
        at_least = max(1, min(at_least, want))
        deadline = time.time() + timeout
        with self.cv:
            self.waiting += 1
            try:
                while len(self.free) < at_least:
                    if (stop is not None and stop.is_set()) or time.time() > deadline:
                        raise KubeMLException("no free workers", 503)
                    if self.reclaimers:
                        self.cv.release()
                        try:
                            for r in self.reclaimers:
                                r()
                        finally:
                            self.cv.acquire()
                        if len(self.free) >= at_least:
                            break
                    self.cv.wait(0.5)
            finally:
                self.waiting -= 1
            got = self.free[:want]
            self.free = self.free[want:]
            return got

    def n_free(self) -> int:
        with self.cv:
            return len(self.free)

    def release(self, ids: List[int]):
        with self.cv:
            for i in ids:
                if i not in self.free:
                    self.free.append(i)
            self.free.sort()
            self.cv.notify_all()


class ParameterServer:
    def __init__(self, store_dir: str, n_workers: int, use_gpu: bool, metrics: Optional[Metrics] = None,
                 scheduler=None, max_parallelism: int = -1, freeze_parallelism: bool = False,
                 worker_env: Optional[Dict[str, str]] = None, task_timeout: float = 3600.0,
                 worker_threads: int = 1, n_gpus: Optional[int] = None):
        self.store_dir = store_dir
        self.n_gpus = n_gpus          # physical GPUs: slot s runs on GPU s % n_gpus
        self.inventory = Inventory(n_workers, use_gpu)
        self.use_gpu = use_gpu
        self.metrics = metrics or Metrics()
        self.scheduler = scheduler
        self.max_parallelism = n_workers if max_parallelism <= 0 else min(max_parallelism, n_workers)
        self.freeze = freeze_parallelism
        self.worker_env = dict(worker_env or {})
        self.task_timeout = task_timeout
        self.worker_threads = worker_threads
        self.functions = FunctionStore(store_dir)
        self.histories = HistoryStore(store_dir)
        self.jobs: Dict[str, TrainJob] = {}
        self.alloc: Dict[str, List[int]] = {}
        self._lock = threading.RLock()
        self._infer_pool: Optional[WorkerPool] = None
        self._infer_lock = threading.Lock()
        self.finished: Dict[str, Optional[str]] = {}
        self.inventory.reclaimers.append(self._reclaim_infer)

    # ------------------------------------------------------------------ pools
    def _pool_for(self, job: TrainJob) -> WorkerPool:
        """Slots for a job's worker pool.  A static job takes exactly its parallelism; an
        elastic one takes its parallelism at least and up to ``max_parallelism`` when
        free (idle GPUs stay warm for scale-ups, the analogue of the reference's Fission
        pool), and gives slots back above ``_shrink_to`` (recovery, or another job
        waiting: see TrainJob._maybe_release_idle)."""
        with self._lock:
            ids = self.alloc.get(job.id)
        shrink = getattr(job, "_shrink_to", None)
        job._shrink_to = None
        if ids is None:
            p = max(1, min(job.parallelism, self.max_parallelism))
            want = p if job.static else self.max_parallelism
            ids = self.inventory.acquire(want, stop=job._stop, at_least=p)
            with self._lock:
                self.alloc[job.id] = ids
        elif shrink is not None and shrink < len(ids):
            keep, drop = ids[:shrink], ids[shrink:]
            self.inventory.release(drop)
            ids = keep
            with self._lock:
                self.alloc[job.id] = ids
        pool = WorkerPool(len(ids), self.use_gpu, self.store_dir, gpu_ids=ids, env=self.worker_env,
                          timeout=self.task_timeout, threads=self.worker_threads, n_gpus=self.n_gpus)
        return pool.start()

    # ------------------------------------------------------------------ API (ps/api.go)
    def start_task(self, task: TrainTask) -> str:
        fn = task.request.function_name
        if not self.functions.exists(fn):
            raise NotFoundError(f"function {fn}")
        with self._lock:
            if task.job.id in self.jobs:
                raise BadRequestError(f"job {task.job.id} already running")
            job = TrainJob(task, code_path=self.functions.code_path(fn), store_dir=self.store_dir,
                           pool_factory=self._pool_for, on_metrics=self._job_metrics, on_finish=self.job_finished,
                           request_update=(self.scheduler.update_job if self.scheduler else None),
                           history_store=self.histories, max_parallelism=self.max_parallelism,
                           freeze_parallelism=self.freeze, task_timeout=self.task_timeout,
                           inventory=self.inventory)
            self.jobs[task.job.id] = job
        self.metrics.task_started("train")
        job.start()
        return task.job.id

    def update_task(self, job_id: str, state: JobState):
        job = self._job(job_id)
        job.update(state)

    def update_metrics(self, job_id: str, m: MetricUpdate):
        self.metrics.update(job_id, m)

    def _job_metrics(self, job_id: str, m: MetricUpdate, job: TrainJob):
        self.update_metrics(job_id, m)
        self.metrics.update_extra(job_id, images_per_second=job.images_per_second,
                                  allreduce_seconds=getattr(job, "last_sync_seconds", None),
                                  hbm_bytes=getattr(job, "last_hbm", None))

    def job_finished(self, job_id: str, err: Optional[str] = None):
        """reference finishJob (api.go:266-327): clear metrics, notify the scheduler."""
        with self._lock:
            self.jobs.pop(job_id, None)
            ids = self.alloc.pop(job_id, [])
            self.finished[job_id] = err
        self.inventory.release(ids)
        self.metrics.clear(job_id)
        self.metrics.task_finished("train")
        if err:
            log.error("job %s finished with error: %s", job_id, err)
        if self.scheduler is not None:
            try:
                self.scheduler.finish_job(job_id)
            except Exception as e:
                log.warning("scheduler finish failed: %r", e)

    def stop_task(self, job_id: str):
        self._job(job_id).stop()

    def list_tasks(self) -> List[TrainTask]:
        with self._lock:
            out = []
            for j in self.jobs.values():
                j.task.job.state.parallelism = j.parallelism
                out.append(j.task)
            return out

    def _job(self, job_id: str) -> TrainJob:
        with self._lock:
            j = self.jobs.get(job_id)
        if j is None:
            raise NotFoundError(f"job {job_id}")
        return j

    def wait(self, job_id: str, timeout: Optional[float] = None) -> Optional[str]:
        """Block until a job finishes (tests / CLI ``--wait``); returns its error."""
        with self._lock:
            j = self.jobs.get(job_id)
        if j is not None and not j.done.wait(timeout):
            raise TimeoutError(job_id)
        t_end = time.time() + 5
        while job_id not in self.finished and time.time() < t_end:
            time.sleep(0.01)
        return self.finished.get(job_id)

    # ------------------------------------------------------------------ inference
    def infer(self, req: InferRequest):
        if not req.model_id:
            raise BadRequestError("model_id is required")
        if not req.data:
            raise BadRequestError("Data not present in request")
        hist = self.histories.get(req.model_id)
        ck = ckpt_path(self.store_dir, req.model_id)
        if not os.path.exists(ck):
            raise NotFoundError(f"checkpoint of model {req.model_id}")
        fn = hist.task.function_name
        if not self.functions.exists(fn):
            raise NotFoundError(f"function {fn}")
        with self._infer_lock:
            if self._infer_pool is None or self._infer_pool.broken:
                ids = self.inventory.acquire(1)
                self._infer_ids = ids
                self._infer_pool = WorkerPool(1, self.use_gpu, self.store_dir, gpu_ids=ids, env=self.worker_env,
                                              timeout=self.task_timeout, n_gpus=self.n_gpus).start()
                self.metrics.task_started("inference")
            msg = {"op": "task", "kind": "infer", "job": f"infer-{req.model_id}", "function": fn,
                   "code_path": self.functions.code_path(fn), "N": 1, "K": -1, "batch_size": hist.task.batch_size,
                   "lr": hist.task.lr, "epoch": 1, "data": req.data, "checkpoint": ck}
            rep = self._infer_pool.call(0, msg)
        if not rep.get("ok"):
            raise KubeMLException(rep.get("error", "inference failed"), int(rep.get("code", 500)))
        return rep["result"]

    def _reclaim_infer(self):
        """A training job is waiting for slots: shut the idle inference pool down (it is
        re-created on the next inference request)."""
        if not self._infer_lock.acquire(blocking=False):
            return
        try:
            if self._infer_pool is not None:
                self._infer_pool.shutdown()
                self._infer_pool = None
                self.inventory.release(getattr(self, "_infer_ids", []))
                self.metrics.task_finished("inference")
        finally:
            self._infer_lock.release()

    def close(self):
        for j in list(self.jobs.values()):
            j.stop()
        with self._infer_lock:
            if self._infer_pool is not None:
                self._infer_pool.shutdown()
                self.inventory.release(getattr(self, "_infer_ids", []))
                self._infer_pool = None
                self.metrics.task_finished("inference")

    # ------------------------------------------------------------------ REST (api.go:335-345)
    def router(self) -> Router:
        r = Router("ps")
        r.add("POST", "/start", lambda q: self.start_task(TrainTask.from_dict(q.json())))
        r.add("POST", "/update/{jobId}", lambda q: self.update_task(q.params["jobId"], JobState.from_dict(q.json()))
              or "")
        r.add("POST", "/metrics/{jobId}",
              lambda q: self.update_metrics(q.params["jobId"], MetricUpdate.from_dict(q.json())) or "")
        r.add("POST", "/finish/{jobId}",
              lambda q: self.job_finished(q.params["jobId"], q.body.decode() or None) or "")
        r.add("DELETE", "/stop/{jobId}", lambda q: self.stop_task(q.params["jobId"]) or "")
        r.add("GET", "/tasks", lambda q: [t.to_dict() for t in self.list_tasks()])
        r.add("GET", "/health", lambda q: "")
        # each TrainJob's own REST surface (reference: one job pod per TrainJob serving
        # ml/pkg/train/api.go:141-149), reached through the PS on this single node
        r.add("GET|POST|DELETE", "/job/{jobId}/{op}", self._job_dispatch)
        return r

    def _job_dispatch(self, q):
        from ..api.errors import NotFoundError
        job = self.jobs.get(q.params["jobId"])
        if job is None:
            raise NotFoundError(f"job {q.params['jobId']}")
        jr = getattr(job, "_router", None)
        if jr is None:
            jr = job._router = job.router()
        return jr.dispatch(q.method, "/" + q.params["op"], q.query, q.headers, q.body)

    def metrics_router(self) -> Router:
        from .http import Response
        r = Router("metrics")
        r.add("GET", "/metrics", lambda q: Response(self.metrics.exposition(), 200, self.metrics.content_type))
        r.add("GET", "/health", lambda q: "")
        return r
