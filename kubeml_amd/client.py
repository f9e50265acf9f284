"""Python client of the controller REST API (reference Go SDK ml/pkg/controller/client:
``V1Interface{Networks, Datasets, Histories, Tasks}``, client.go:11-59, v1/*.go).

The controller URL comes from ``KUBEML_CONTROLLER_URL`` (default
``http://127.0.0.1:10100``) instead of k8s Service discovery (client/util.go:17-65).
"""
from __future__ import annotations

import os
from typing import Any, List, Optional

from .api.types import DatasetSummary, History, InferRequest, TrainRequest, TrainTask
from .control.http import call, multipart_encode


class _Sub:
    def __init__(self, c: "KubemlClient"):
        self.c = c


class Networks(_Sub):
    def train(self, req: TrainRequest) -> str:
        return self.c._call("POST", "/train", json_body=req.to_dict()).strip()

    def infer(self, req: InferRequest) -> Any:
        return self.c._call("POST", "/infer", json_body=req.to_dict())


class Datasets(_Sub):
    def create(self, name: str, train_data: str, train_labels: str, test_data: str, test_labels: str):
        fields = {}
        for key, path in (("x-train", train_data), ("y-train", train_labels), ("x-test", test_data),
                          ("y-test", test_labels)):
            with open(path, "rb") as f:
                fields[key] = (os.path.basename(path), f.read())
        body, ctype = multipart_encode(fields)
        return self.c._call("POST", f"/dataset/{name}", data=body, headers={"Content-Type": ctype})

    def delete(self, name: str):
        return self.c._call("DELETE", f"/dataset/{name}")

    def get(self, name: str) -> DatasetSummary:
        return DatasetSummary.from_dict(self.c._call("GET", f"/dataset/{name}"))

    def list(self) -> List[DatasetSummary]:
        return [DatasetSummary.from_dict(d) for d in self.c._call("GET", "/dataset")]


class Histories(_Sub):
    def get(self, job_id: str) -> History:
        return History.from_dict(self.c._call("GET", f"/history/{job_id}"))

    def delete(self, job_id: str):
        return self.c._call("DELETE", f"/history/{job_id}")

    def list(self) -> List[History]:
        return [History.from_dict(h) for h in self.c._call("GET", "/history")]

    def prune(self):
        return self.c._call("DELETE", "/history")


class Tasks(_Sub):
    def list(self) -> List[TrainTask]:
        return [TrainTask.from_dict(t) for t in self.c._call("GET", "/tasks")]

    def stop(self, job_id: str):
        return self.c._call("DELETE", f"/tasks/{job_id}")

    def status(self, job_id: str) -> dict:
        return self.c._call("GET", f"/jobs/{job_id}")


class Functions(_Sub):
    def create(self, name: str, code_path: str):
        with open(code_path, "rb") as f:
            code = f.read()
        return self.c._call("POST", f"/function/{name}", data=code, headers={"Content-Type": "text/x-python"})

    def delete(self, name: str):
        return self.c._call("DELETE", f"/function/{name}")

    def list(self) -> List[dict]:
        return self.c._call("GET", "/function")


class KubemlClient:
    def __init__(self, url: Optional[str] = None, timeout: float = 3600.0):
        self.url = (url or os.environ.get("KUBEML_CONTROLLER_URL") or "http://127.0.0.1:10100").rstrip("/")
        self.timeout = timeout
        self.networks = Networks(self)
        self.datasets = Datasets(self)
        self.histories = Histories(self)
        self.tasks = Tasks(self)
        self.functions = Functions(self)

    def _call(self, method, path, **kw):
        return call(method, self.url + path, timeout=self.timeout, **kw)

    def logs(self, job_id: str, since: int = 0) -> bytes:
        return call("GET", f"{self.url}/logs/{job_id}?since={since}", raw=True, timeout=self.timeout)

    def health(self) -> bool:
        try:
            self._call("GET", "/health")
            return True
        except Exception:
            return False
