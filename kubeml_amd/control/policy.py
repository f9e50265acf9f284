"""Scheduling policies — thin binding over the native policy core (csrc/runtime/policy.cpp).

``ThroughputPolicy`` is the reference's ThroughputBasedPolicy (ml/pkg/scheduler/policy.go)
with the thresholds 1.05 / 1.2, clamped to [1, max_parallelism] and thread-safe.
``SchedulerPolicy`` is the pluggable interface (policy.go:18-22).
"""
from __future__ import annotations

from typing import Tuple

from ..api.types import SCALE_DOWN_THRESHOLD, SCALE_UP_THRESHOLD


class SchedulerPolicy:
    def decide(self, job_id: str, default: int, parallelism: int, elapsed: float) -> Tuple[int, str]:
        raise NotImplementedError

    def finish(self, job_id: str):
        raise NotImplementedError


class ThroughputPolicy(SchedulerPolicy):
    def __init__(self, max_parallelism: int = 8, min_parallelism: int = 1, scale_up: float = SCALE_UP_THRESHOLD,
                 scale_down: float = SCALE_DOWN_THRESHOLD):
        from .._native import RT
        self._rt = RT
        self._h = RT.raw("kml_policy_new", float(scale_up), float(scale_down), int(min_parallelism),
                         int(max_parallelism))
        if not self._h:
            raise RuntimeError("native policy allocation failed")
        self.max_parallelism = max_parallelism

    def set_bounds(self, min_p: int, max_p: int):
        self._rt.raw("kml_policy_set_bounds", self._h, int(min_p), int(max_p))
        self.max_parallelism = max_p

    def decide(self, job_id, default, parallelism, elapsed):
        import ctypes
        op = ctypes.c_int(0)
        p = self._rt.raw("kml_policy_decide", self._h, job_id.encode(), int(default), int(parallelism),
                         float(elapsed), ctypes.addressof(op))
        return int(p), ("create" if op.value == 0 else "update")

    def finish(self, job_id):
        self._rt.raw("kml_policy_finish", self._h, job_id.encode())

    def reference_time(self, job_id) -> float:
        return float(self._rt.raw("kml_policy_reference_time", self._h, job_id.encode()))

    def __del__(self):
        try:
            self._rt.raw("kml_policy_free", self._h)
        except Exception:
            pass


class StaticPolicy(SchedulerPolicy):
    """Keeps the requested parallelism (``--static``)."""

    def __init__(self, max_parallelism: int = 8):
        self.max_parallelism = max_parallelism
        self._seen = set()

    def decide(self, job_id, default, parallelism, elapsed):
        if job_id not in self._seen:
            self._seen.add(job_id)
            return max(1, min(default, self.max_parallelism)), "create"
        return parallelism, "update"

    def finish(self, job_id):
        self._seen.discard(job_id)


class ScriptedPolicy(SchedulerPolicy):
    """Deterministic policy: the i-th decision for a job returns ``seq[i]`` (the last
    value repeats), clamped to [1, max_parallelism].  Drives reproducible elastic
    experiments (north-star config 4: VGG-16 at P = 2 -> 4 -> 8) and resize tests;
    select it with ``KUBEML_POLICY=scripted:2,4,8``."""

    def __init__(self, seq, max_parallelism: int = 8):
        self.seq = [int(x) for x in seq] or [1]
        self.max_parallelism = max_parallelism
        self._n = {}
        import threading
        self._lock = threading.Lock()

    def decide(self, job_id, default, parallelism, elapsed):
        with self._lock:
            i = self._n.get(job_id, 0)
            self._n[job_id] = i + 1
        p = self.seq[min(i, len(self.seq) - 1)]
        return max(1, min(p, self.max_parallelism)), ("create" if i == 0 else "update")

    def finish(self, job_id):
        with self._lock:
            self._n.pop(job_id, None)


def policy_from_spec(spec: str, max_parallelism: int) -> SchedulerPolicy:
    """``throughput`` (default) | ``static`` | ``scripted:p1,p2,...``."""
    spec = (spec or "throughput").strip()
    if spec == "throughput":
        return ThroughputPolicy(max_parallelism=max_parallelism)
    if spec == "static":
        return StaticPolicy(max_parallelism=max_parallelism)
    if spec.startswith("scripted:"):
        return ScriptedPolicy(spec.split(":", 1)[1].split(","), max_parallelism=max_parallelism)
    raise ValueError(f"unknown policy {spec!r}")
