"""Controller — the public REST gateway (reference ml/pkg/controller/*.go).

Routes (api.go:16-42):

=========================  ===========================================================
``POST /train``            TrainRequest → plain-text job id (via the scheduler)
``POST /infer``            InferRequest → predictions (scheduler → PS → worker)
``GET /dataset/{name}``    DatasetSummary, 404 if missing
``POST|DELETE /dataset/…`` storage service (multipart ``x-train,y-train,x-test,y-test``)
``GET /dataset``           [DatasetSummary]
``GET /tasks``             [TrainTask]; ``DELETE /tasks/{jobId}`` stops one
``GET|DELETE /history/…``  one history; ``GET /history`` list; ``DELETE /history`` prune
``GET /health``            liveness
=========================  ===========================================================

Additions (the reference used Fission / kubectl for these): ``GET|POST|DELETE
/function[/{name}]`` (function registry), ``GET /logs/{jobId}`` (job log, ``?since=``
byte offset for follow mode), ``GET /jobs/{jobId}`` (status incl. finish error).
"""
from __future__ import annotations

import os

from ..api.errors import KubeMLException, NotFoundError
from ..api.types import InferRequest, TrainRequest
from ..store import service as storage
from ..store.functions import FunctionStore
from ..store.history import HistoryStore
from ..store.shards import ShardStore
from .http import Response, Router


class Controller:
    def __init__(self, store_dir: str, scheduler, ps, shards: ShardStore = None, histories: HistoryStore = None,
                 functions: FunctionStore = None):
        self.store_dir = store_dir
        self.scheduler = scheduler
        self.ps = ps
        self.shards = shards or ShardStore(store_dir)
        self.histories = histories or HistoryStore(store_dir)
        self.functions = functions or FunctionStore(store_dir)

    # --- network (networkApi.go) ---------------------------------------------------
    def train(self, req: TrainRequest) -> str:
        opts = req.options
        if getattr(opts, "sync", "") == "grad" and (int(opts.k) != 1 or not opts.static_parallelism):
            # persistent (sharded) optimizer state across K = 1 rounds: an elastic resize would start
            # new workers from zero moments and move shard ownership; the CLI checks too
            from ..api.errors import KubeMLException
            raise KubeMLException("sync='grad' needs k = 1 and static_parallelism", 400)
        if not self.shards.exists(req.dataset):
            raise NotFoundError(f"dataset {req.dataset}")
        if not self.functions.exists(req.function_name):
            raise NotFoundError(f"function {req.function_name}")
        return self.scheduler.submit_train(req)

    def infer(self, req: InferRequest):
        return self.scheduler.infer(req)

    # --- tasks (tasksApi.go) -------------------------------------------------------
    def tasks(self):
        return [t.to_dict() for t in self.ps.list_tasks()]

    def stop_task(self, job_id: str):
        self.ps.stop_task(job_id)

    def job_status(self, job_id: str):
        if self.scheduler.is_pending(job_id):
            return {"id": job_id, "state": "running", "queued": True, "parallelism": 0}
        running = {t.job.id: t for t in self.ps.list_tasks()}
        if job_id in running:
            t = running[job_id]
            return {"id": job_id, "state": "running", "parallelism": t.job.state.parallelism}
        if job_id in self.ps.finished:
            err = self.ps.finished[job_id]
            return {"id": job_id, "state": "failed" if err else "finished", "error": err}
        if self.histories.exists(job_id):
            return {"id": job_id, "state": "finished", "error": None}
        if job_id in self.scheduler.failed:
            return {"id": job_id, "state": "failed", "error": self.scheduler.failed[job_id]}
        raise NotFoundError(f"job {job_id}")

    # --- logs ----------------------------------------------------------------------
    def logs(self, job_id: str, since: int = 0):
        p = os.path.join(self.store_dir, "logs", f"{job_id}.log")
        if not os.path.exists(p):
            raise NotFoundError(f"logs of job {job_id}")
        with open(p, "rb") as f:
            f.seek(since)
            data = f.read()
        return Response(data, 200, "text/plain; charset=utf-8")

    # --- functions -----------------------------------------------------------------
    def create_function(self, name: str, code: bytes):
        from dataclasses import asdict
        return asdict(self.functions.create(name, code))

    def router(self) -> Router:
        from dataclasses import asdict
        r = Router("controller")
        r.add("POST", "/train", lambda q: Response(self.train(TrainRequest.from_dict(q.json())), 200, "text/plain"))
        r.add("POST", "/infer", lambda q: self.infer(InferRequest.from_dict(q.json())))
        r.add("GET", "/dataset/{name}", lambda q: self.shards.summary(q.params["name"]).to_dict())
        st = storage.router(self.shards)
        r.add("POST", "/dataset/{name}",
              lambda q: st.dispatch("POST", q.path, q.query, q.headers, q.body))
        r.add("DELETE", "/dataset/{name}",
              lambda q: st.dispatch("DELETE", q.path, q.query, q.headers, q.body))
        r.add("GET", "/dataset", lambda q: [s.to_dict() for s in self.shards.list()])
        r.add("GET", "/tasks", lambda q: self.tasks())
        r.add("DELETE", "/tasks/{jobId}", lambda q: self.stop_task(q.params["jobId"]) or "")
        r.add("GET", "/jobs/{jobId}", lambda q: self.job_status(q.params["jobId"]))
        r.add("GET", "/history/{taskId}", lambda q: self.histories.get(q.params["taskId"]).to_dict())
        r.add("DELETE", "/history/{taskId}", lambda q: self.histories.delete(q.params["taskId"]) or "")
        r.add("GET", "/history", lambda q: [h.to_dict() for h in self.histories.list()])
        r.add("DELETE", "/history", lambda q: {"deleted": self.histories.prune()})
        r.add("GET", "/function", lambda q: [asdict(f) for f in self.functions.list()])
        r.add("GET", "/function/{name}", lambda q: asdict(self.functions.get(q.params["name"])))
        r.add("POST", "/function/{name}", lambda q: self.create_function(q.params["name"], q.body))
        r.add("DELETE", "/function/{name}", lambda q: self.functions.delete(q.params["name"]) or "")
        r.add("GET", "/logs/{jobId}", lambda q: self.logs(q.params["jobId"], int(q.query.get("since", 0) or 0)))
        r.add("GET", "/health", lambda q: "")
        return r
