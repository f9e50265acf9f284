"""Wire types of the control plane — same JSON field names as the reference.

Mirrors ml/pkg/api/types.go:13-111 field-for-field (including the reference's
``validations_loss`` spelling in MetricUpdate, types.go:85-91) so existing clients,
the experiments harness and stored histories interoperate.
"""
from __future__ import annotations

import json
from dataclasses import asdict, dataclass, field, fields
from typing import Any, Dict, List, Optional


class _Json:
    """to_dict / from_dict with nested dataclasses and tolerant of unknown keys."""

    _OMIT_EMPTY: tuple = ()  # extension fields left out of the wire form when unset

    def to_dict(self) -> Dict[str, Any]:
        out = {}
        for f in fields(self):
            v = getattr(self, f.name)
            if f.name in self._OMIT_EMPTY and not v:
                continue
            if isinstance(v, _Json):
                v = v.to_dict()
            elif isinstance(v, list):
                v = [x.to_dict() if isinstance(x, _Json) else x for x in v]
            out[f.name] = v
        return out

    def to_json(self) -> str:
        return json.dumps(self.to_dict())

    @classmethod
    def from_dict(cls, d: Optional[Dict[str, Any]]):
        d = d or {}
        kw = {}
        for f in fields(cls):
            if f.name not in d:
                continue
            v = d[f.name]
            t = f.type if not isinstance(f.type, str) else _TYPES.get(f.type)
            if isinstance(t, type) and issubclass(t, _Json) and isinstance(v, dict):
                v = t.from_dict(v)
            kw[f.name] = v
        return cls(**kw)

    @classmethod
    def from_json(cls, s):
        return cls.from_dict(json.loads(s) if isinstance(s, (str, bytes)) else s)


@dataclass
class TrainOptions(_Json):
    default_parallelism: int = 2
    static_parallelism: bool = False
    validate_every: int = 0
    k: int = -1
    goal_accuracy: float = 100.0
    resume_from: str = ""   # extension: continue a finished/failed job from its checkpoint
    # extension: "grad" = K=1 rounds as synchronous data parallelism with PERSISTENT optimizer
    # state (Adam moments, momentum carry across rounds).  A deliberate departure from the
    # reference, which rebuilds the optimizer every round (network.py:208-217) — with Adam
    # that makes every step a first step.  "" = the reference semantics.
    sync: str = ""
    _OMIT_EMPTY = ("resume_from", "sync")


@dataclass
class TrainRequest(_Json):
    model_type: str = "example"
    batch_size: int = 64
    epochs: int = 1
    dataset: str = ""
    lr: float = 0.01
    function_name: str = ""
    options: TrainOptions = field(default_factory=TrainOptions)


@dataclass
class InferRequest(_Json):
    model_id: str = ""
    data: List[Any] = field(default_factory=list)


@dataclass
class JobState(_Json):
    parallelism: int = 0
    elapsed_time: float = 0.0


@dataclass
class JobInfo(_Json):
    id: str = ""
    state: JobState = field(default_factory=JobState)


@dataclass
class TrainTask(_Json):
    request: TrainRequest = field(default_factory=TrainRequest)
    job: JobInfo = field(default_factory=JobInfo)


@dataclass
class JobHistory(_Json):
    validation_loss: List[float] = field(default_factory=list)
    accuracy: List[float] = field(default_factory=list)
    train_loss: List[float] = field(default_factory=list)
    parallelism: List[float] = field(default_factory=list)
    epoch_duration: List[float] = field(default_factory=list)
    # extension (omitted from the wire form when empty): how each epoch synchronised the
    # workers — "kavg" (reference K-AVG), "kavg-async-staleness1", "grad-allreduce" (K=1 DP)
    sync_mode: List[str] = field(default_factory=list)
    _OMIT_EMPTY = ("sync_mode",)


@dataclass
class MetricUpdate(_Json):
    validations_loss: float = 0.0  # sic: reference spelling (types.go:86)
    accuracy: float = 0.0
    train_loss: float = 0.0
    parallelism: float = 0.0
    epoch_duration: float = 0.0


@dataclass
class History(_Json):
    id: str = ""
    task: TrainRequest = field(default_factory=TrainRequest)
    data: JobHistory = field(default_factory=JobHistory)


@dataclass
class DatasetSummary(_Json):
    name: str = ""
    train_set_size: int = 0
    test_set_size: int = 0


_TYPES = {c.__name__: c for c in (TrainOptions, TrainRequest, InferRequest, JobState, JobInfo, TrainTask,
                                  JobHistory, MetricUpdate, History, DatasetSummary)}

# Constants of the reference (ml/pkg/api/const.go, python/kubeml/kubeml/util.py:10)
DEFAULT_PARALLELISM = 5
STORAGE_SUBSET_SIZE = 64
MAX_BATCH = 1024
SCALE_UP_THRESHOLD = 1.05
SCALE_DOWN_THRESHOLD = 1.2
