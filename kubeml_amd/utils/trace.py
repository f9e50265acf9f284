"""Chrome-trace spans (``KUBEML_TRACE=1``) — the reference has no tracing at all
(ad-hoc ``time.Since`` logs in job.go:307-327 only).

Each process records complete events (``ph: "X"``) with wall-clock microseconds; on
GPU workers a span can also be closed on the device timeline (``cuda=True`` syncs the
current stream at both ends, so use it only in diagnostic runs).  ``flush()`` writes
``<dir>/<name>-pid<pid>.json`` loadable in chrome://tracing / Perfetto.

Span names used by the runtime: ``task:<kind>``, ``load``, ``iteration``,
``average``, ``broadcast``, ``validate``, ``epoch``, ``sync-wait``.

Device timeline (SURVEY §5.1 "comm/compute overlap timeline"): :func:`gpu_span` takes
two timing events recorded on a HIP stream and places the span on a per-track row
(``gpu:compute``, ``gpu:comm``) of the same trace, in host-clock microseconds: the first
device mark is anchored to the host clock once (event synchronise), every later event
is placed by its device-side elapsed time from that anchor.  Events resolve lazily at
:func:`flush`, so marking costs nothing on the hot path but an event record.
"""
from __future__ import annotations

import json
import os
import threading
import time
from contextlib import contextmanager
from typing import List, Optional

_enabled = os.environ.get("KUBEML_TRACE", "0").lower() in ("1", "true", "yes", "on")
_events: List[dict] = []
_lock = threading.Lock()
_meta = {"rank": None, "name": "kubeml"}


def enabled() -> bool:
    return _enabled


def enable(on: bool = True):
    global _enabled
    _enabled = on


def set_process(name: str, rank: Optional[int] = None):
    _meta["name"] = name
    _meta["rank"] = rank


@contextmanager
def span(name: str, cat: str = "kubeml", cuda: bool = False, **args):
    if not _enabled:
        yield
        return
    if cuda:
        _sync()
    t0 = time.perf_counter_ns()
    try:
        yield
    finally:
        if cuda:
            _sync()
        t1 = time.perf_counter_ns()
        ev = {"name": name, "cat": cat, "ph": "X", "ts": t0 / 1e3, "dur": (t1 - t0) / 1e3,
              "pid": os.getpid(), "tid": threading.get_ident() % 100000, "args": args}
        with _lock:
            _events.append(ev)


def instant(name: str, **args):
    if not _enabled:
        return
    with _lock:
        _events.append({"name": name, "ph": "i", "s": "p", "ts": time.perf_counter_ns() / 1e3, "pid": os.getpid(),
                        "tid": threading.get_ident() % 100000, "args": args})


_gpu = {"anchor": None, "anchor_ns": 0, "pending": []}
_TRACKS = {"gpu:compute": 900001, "gpu:comm": 900002, "gpu:copy": 900003}


def gpu_mark(stream=None):
    """A timing event recorded on ``stream`` (default: current), or None if tracing is off."""
    if not _enabled:
        return None
    import torch
    if _gpu["anchor"] is None:
        a = torch.cuda.Event(enable_timing=True)
        a.record(torch.cuda.current_stream())
        a.synchronize()
        _gpu["anchor"], _gpu["anchor_ns"] = a, time.perf_counter_ns()
    e = torch.cuda.Event(enable_timing=True)
    e.record(stream if stream is not None else torch.cuda.current_stream())
    return e


def gpu_span(name: str, start, end, track: str = "gpu:compute", **args):
    """Device-timeline span between two :func:`gpu_mark` events."""
    if not _enabled or start is None or end is None:
        return
    with _lock:
        _gpu["pending"].append((name, start, end, track, args))


def _resolve_gpu():
    pend = _gpu["pending"]
    if not pend:
        return []
    anchor, a_ns = _gpu["anchor"], _gpu["anchor_ns"]
    out = []
    for name, e0, e1, track, args in pend:
        e1.synchronize()
        t0 = a_ns / 1e3 + anchor.elapsed_time(e0) * 1e3
        t1 = a_ns / 1e3 + anchor.elapsed_time(e1) * 1e3
        out.append({"name": name, "cat": "gpu", "ph": "X", "ts": t0, "dur": max(t1 - t0, 0.0), "pid": os.getpid(),
                    "tid": _TRACKS.get(track, 900009), "args": args})
    pend.clear()
    return out


def _sync():
    try:
        import torch
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.current_stream().synchronize()
    except Exception:
        pass


def events() -> List[dict]:
    with _lock:
        return list(_events)


_FLUSHES = 0


def flush(directory: Optional[str] = None, clear: bool = True) -> Optional[str]:
    """Write collected events; returns the file path (None if nothing recorded)."""
    try:
        gevs = _resolve_gpu()
    except Exception:
        gevs = []
    with _lock:
        evs = list(_events) + gevs
        if clear:
            _events.clear()
    if not evs:
        return None
    directory = directory or os.environ.get("KUBEML_TRACE_DIR", os.path.join(os.path.expanduser("~/.kubeml"), "traces"))
    os.makedirs(directory, exist_ok=True)
    rank = _meta["rank"]
    name = _meta["name"] + (f"-rank{rank}" if rank is not None else "")
    meta = [{"name": "process_name", "ph": "M", "pid": os.getpid(), "args": {"name": name}}]
    meta += [{"name": "thread_name", "ph": "M", "pid": os.getpid(), "tid": tid, "args": {"name": tr}}
             for tr, tid in _TRACKS.items()]
    # one file per flush (workers flush after every task): earlier tasks' spans are kept
    global _FLUSHES
    _FLUSHES += 1
    path = os.path.join(directory, f"{name}-pid{os.getpid()}-{_FLUSHES:04d}.json")
    with open(path, "w") as f:
        json.dump({"traceEvents": meta + evs, "displayTimeUnit": "ms"}, f)
    return path
