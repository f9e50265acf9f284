"""Training-history store (the reference's Mongo ``kubeml.history`` collection).

Reference: the TrainJob writes ``History{_id: jobId, task: TrainRequest, data:
JobHistory}`` at the end of training (ml/pkg/train/util.go:247-280); the controller
lists / gets / deletes / prunes them (ml/pkg/controller/historyApi.go:14-111).

Here: one JSON document per job under ``<store>/history/<jobId>.json`` written
atomically, same schema and field names (``id`` is the document's ``_id``).
Histories are also updated after every epoch (not only at job end) so a crashed
job leaves its partial history behind and ``kubeml history get`` works mid-run.
"""
from __future__ import annotations

import os
import threading
from typing import List

from ..api.errors import NotFoundError
from ..api.types import History
from ._fs import check_name, read_json, write_json


class HistoryStore:
    def __init__(self, root: str):
        self.root = os.path.join(root, "history")
        os.makedirs(self.root, exist_ok=True)
        self._lock = threading.Lock()

    def _path(self, job_id: str) -> str:
        return os.path.join(self.root, check_name(job_id, "job id") + ".json")

    def save(self, h: History):
        with self._lock:
            write_json(self._path(h.id), h.to_dict())

    def exists(self, job_id: str) -> bool:
        return os.path.exists(self._path(job_id))

    def get(self, job_id: str) -> History:
        p = self._path(job_id)
        if not os.path.exists(p):
            raise NotFoundError(f"history {job_id}")
        return History.from_dict(read_json(p))

    def list(self) -> List[History]:
        out = []
        for f in sorted(os.listdir(self.root)):
            if f.endswith(".json") and not f.startswith("."):
                try:
                    out.append(History.from_dict(read_json(os.path.join(self.root, f))))
                except (OSError, ValueError):
                    continue
        return out

    def delete(self, job_id: str):
        with self._lock:
            p = self._path(job_id)
            if not os.path.exists(p):
                raise NotFoundError(f"history {job_id}")
            os.unlink(p)

    def prune(self) -> int:
        n = 0
        with self._lock:
            for f in os.listdir(self.root):
                if f.endswith(".json"):
                    os.unlink(os.path.join(self.root, f))
                    n += 1
        return n
