"""HTTP clients of the internal roles (reference Go clients):

* :class:`SchedulerClient` — ml/pkg/scheduler/client/client.go:36-122
  (``UpdateJob`` POST /job, ``FinishJob`` DELETE /finish/{id}, ``SubmitTrainTask``
  POST /train → id, ``SubmitInferenceTask`` POST /infer)
* :class:`PSClient` — ml/pkg/ps/client/client.go:33-160 (``StopTask``, ``ListTasks``,
  ``UpdateTask``, ``StartTask``, ``UpdateMetrics``, ``JobFinished``)
* :class:`JobClient` — ml/pkg/train/client/client.go:23-107 (``Stop``, ``UpdateTask``,
  ``StartTask``) addressed at a job's REST endpoint.

Inside one ``kubeml-server`` process the roles call each other directly; these are
for split deployments (``--role``) and external tooling.
"""
from __future__ import annotations

from typing import List, Optional

from ..api.types import InferRequest, JobState, MetricUpdate, TrainRequest, TrainTask
from .http import call


class SchedulerClient:
    def __init__(self, url: str = "http://127.0.0.1:10200"):
        self.url = url.rstrip("/")

    def update_job(self, task: TrainTask):
        call("POST", f"{self.url}/job", json_body=task.to_dict())

    def finish_job(self, job_id: str):
        call("DELETE", f"{self.url}/finish/{job_id}")

    def submit_train_task(self, req: TrainRequest) -> str:
        return call("POST", f"{self.url}/train", json_body=req.to_dict())

    def submit_inference_task(self, req: InferRequest):
        return call("POST", f"{self.url}/infer", json_body=req.to_dict())


class PSClient:
    def __init__(self, url: str = "http://127.0.0.1:10300"):
        self.url = url.rstrip("/")

    def stop_task(self, job_id: str):
        call("DELETE", f"{self.url}/stop/{job_id}")

    def list_tasks(self) -> List[TrainTask]:
        return [TrainTask.from_dict(t) for t in call("GET", f"{self.url}/tasks")]

    def update_task(self, job_id: str, state: JobState):
        call("POST", f"{self.url}/update/{job_id}", json_body=state.to_dict())

    def start_task(self, task: TrainTask):
        return call("POST", f"{self.url}/start", json_body=task.to_dict())

    def update_metrics(self, job_id: str, m: MetricUpdate):
        call("POST", f"{self.url}/metrics/{job_id}", json_body=m.to_dict())

    def job_finished(self, job_id: str, err: Optional[str] = None):
        call("POST", f"{self.url}/finish/{job_id}", data=(err or "").encode(),
             headers={"Content-Type": "text/plain"})


class JobClient:
    def __init__(self, url: str):
        self.url = url.rstrip("/")

    def stop(self):
        call("DELETE", f"{self.url}/stop")

    def update_task(self, state: JobState):
        call("POST", f"{self.url}/update", json_body=state.to_dict())

    def start_task(self, task: TrainTask):
        call("POST", f"{self.url}/start", json_body=task.to_dict())

    def health(self) -> bool:
        try:
            call("GET", f"{self.url}/health")
            return True
        except Exception:
            return False
