"""Scheduler — FIFO task queue + elastic parallelism policy (reference
ml/pkg/scheduler/{scheduler.go, api.go, queue.go, policy.go}).

* ``submit_train`` (``POST /train``) mints an 8-character job id (util.go:8-10) and
  queues the task (api.go:78-116);
* the queue is served every 10 ms (scheduler.go:48-89): the policy decides the
  parallelism; first sight → ``PS.start_task`` (create), later → ``PS.update_task``;
* ``update_job`` (``POST /job``) is what a TrainJob calls at the end of each epoch;
* ``finish_job`` (``DELETE /finish/{id}``) forgets the job's timing state;
* ``infer`` (``POST /infer``) forwards to the PS, which runs it on a resident worker
  against the job's checkpoint (the reference hard-coded function ``"network"`` and
  never loaded weights, api.go:119-162 — fixed here).

The decision output is the next epoch's worker count, i.e. which RCCL
sub-communicator of the job's world the workers use.
"""
from __future__ import annotations

import collections
import logging
import threading
import uuid
from typing import Optional

from ..api.errors import BadRequestError
from ..api.types import MAX_BATCH, InferRequest, JobInfo, JobState, TrainRequest, TrainTask
from .http import Router
from .policy import SchedulerPolicy, ThroughputPolicy

log = logging.getLogger("kubeml.scheduler")


def create_job_id() -> str:
    return uuid.uuid4().hex[:8]


def validate_request(req: TrainRequest):
    """CLI-side checks of the reference (cli/train.go:150-172), enforced server-side too."""
    if not (0 < int(req.batch_size) <= MAX_BATCH):
        raise BadRequestError(f"batch size must be in (0, {MAX_BATCH}]")
    if int(req.epochs) <= 0:
        raise BadRequestError("epochs must be > 0")
    if float(req.lr) <= 0:
        raise BadRequestError("lr must be > 0")
    if not req.dataset:
        raise BadRequestError("dataset is required")
    if not req.function_name:
        raise BadRequestError("function is required")
    k = int(req.options.k)
    if k == 0 or k < -1:
        raise BadRequestError("K must be -1 (sync once per epoch) or a positive number of local steps")


class Scheduler:
    POLL_S = 0.010

    def __init__(self, ps=None, policy: Optional[SchedulerPolicy] = None, max_parallelism: int = 8):
        self.ps = ps
        self.policy = policy or ThroughputPolicy(max_parallelism=max_parallelism)
        self._q = collections.deque()
        self._pending = set()        # submitted jobs the PS has not taken yet
        self.failed = {}             # job id -> error for jobs the PS refused to start
        self._lock = threading.Lock()
        self._wake = threading.Event()
        self._stop = threading.Event()
        self._t: Optional[threading.Thread] = None

    # ------------------------------------------------------------------ queue (queue.go)
    def _push(self, task: TrainTask):
        with self._lock:
            self._q.append(task)
        self._wake.set()

    def _pop(self) -> Optional[TrainTask]:
        with self._lock:
            return self._q.popleft() if self._q else None

    def queue_length(self) -> int:
        with self._lock:
            return len(self._q)

    # ------------------------------------------------------------------ API
    def submit_train(self, req: TrainRequest) -> str:
        validate_request(req)
        jid = create_job_id()
        with self._lock:
            self._pending.add(jid)
        self._push(TrainTask(request=req, job=JobInfo(id=jid, state=JobState())))
        return jid

    def is_pending(self, job_id: str) -> bool:
        """Submitted but not yet running on the parameter server (status polls between
        ``/train`` and the PS start see the job as queued, not unknown)."""
        with self._lock:
            return job_id in self._pending

    def update_job(self, task: TrainTask):
        self._push(task)

    def finish_job(self, job_id: str):
        self.policy.finish(job_id)

    def infer(self, req: InferRequest):
        return self.ps.infer(req)

    # ------------------------------------------------------------------ loop (scheduler.go:48-89)
    def serve_once(self) -> bool:
        task = self._pop()
        if task is None:
            return False
        p, op = self.policy.decide(task.job.id, int(task.request.options.default_parallelism),
                                   int(task.job.state.parallelism), float(task.job.state.elapsed_time))
        task.job.state.parallelism = p
        try:
            if op == "create":
                self.ps.start_task(task)
            else:
                self.ps.update_task(task.job.id, JobState(parallelism=p, elapsed_time=task.job.state.elapsed_time))
        except Exception as e:
            log.error("error sending task %s to the parameter server: %r", op, e)
            if op == "create":
                self.failed[task.job.id] = repr(e)
        finally:
            with self._lock:
                self._pending.discard(task.job.id)
        return True

    def _loop(self):
        while not self._stop.is_set():
            if not self.serve_once():
                self._wake.wait(self.POLL_S)
                self._wake.clear()

    def start(self) -> "Scheduler":
        self._t = threading.Thread(target=self._loop, name="scheduler", daemon=True)
        self._t.start()
        return self

    def stop(self):
        self._stop.set()
        self._wake.set()

    # ------------------------------------------------------------------ REST (api.go:184-192)
    def router(self) -> Router:
        r = Router("scheduler")
        r.add("POST", "/job", lambda q: self.update_job(TrainTask.from_dict(q.json())) or "")
        r.add("POST", "/train", lambda q: self.submit_train(TrainRequest.from_dict(q.json())))
        r.add("POST", "/infer", lambda q: self.infer(InferRequest.from_dict(q.json())))
        r.add("DELETE", "/finish/{taskId}", lambda q: self.finish_job(q.params["taskId"]) or "")
        r.add("GET", "/health", lambda q: "")
        return r
