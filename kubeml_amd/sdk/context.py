"""Per-invocation task context (replaces the reference's Flask request args).

The reference passes task parameters as query args of the function's HTTP GET
(``/{fn}?task=&jobId=&N=&K=&funcId=&batchSize=&lr=&epoch=``, ml/pkg/train/function.go:44-68)
and user code reads them through ``_KubeArgs.parse()`` (python/kubeml/kubeml/dataset.py:24-78).
A resident worker sets the same fields here before calling the user's ``main()``,
so user functions written for the reference run unchanged.
"""
from __future__ import annotations

import contextvars
from dataclasses import dataclass, field
from typing import Any, Dict, Optional


@dataclass
class TaskContext:
    job_id: str = "local"
    N: int = 1
    K: int = -1
    task: str = "train"
    func_id: int = 0
    lr: float = 0.01
    batch_size: int = 64
    epoch: int = 1
    data: Any = None                   # infer payload (JSON list)
    comm: Any = None                   # kubeml_amd.parallel.comm.Comm of the active workers
    store: Any = None                  # kubeml_amd.store.shards.ShardStore
    store_dir: Optional[str] = None
    device: Any = None                 # torch.device of this worker
    checkpoint: Optional[str] = None   # path of the job's reference-model checkpoint
    extra: Dict[str, Any] = field(default_factory=dict)

    @classmethod
    def from_query(cls, q: Dict[str, Any], **kw) -> "TaskContext":
        """Build from reference-style query args (strings accepted)."""
        def g(name, typ, default):
            v = q.get(name, default)
            return typ(v) if v is not None else default
        return cls(job_id=g("jobId", str, "local"), N=g("N", int, 1), K=g("K", int, -1),
                   task=g("task", str, "train"), func_id=g("funcId", int, 0), lr=g("lr", float, 0.0),
                   batch_size=g("batchSize", int, 0), epoch=g("epoch", int, 1), **kw)


_CURRENT: contextvars.ContextVar = contextvars.ContextVar("kubeml_task", default=None)


def set_task(ctx: TaskContext):
    return _CURRENT.set(ctx)


def reset_task(token):
    _CURRENT.reset(token)


def current_task() -> Optional[TaskContext]:
    return _CURRENT.get()
