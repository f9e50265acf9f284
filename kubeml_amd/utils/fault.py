"""Fault injection for failure-path tests (the reference only *planned*
a "chaos monkey", ml/experiments/README.md:17).

Spec (``KUBEML_FAULT`` or :func:`configure`): ``;``-separated rules
``<action>:<key>=<val>[:<key>=<val>...]`` with actions

* ``kill``  — ``os._exit(17)`` the worker process (simulates a lost GPU/worker),
* ``raise`` — raise ``RuntimeError`` inside the task (function error path),
* ``hang``  — sleep ``secs`` seconds (timeouts / heartbeat tests),

and match keys ``rank``, ``epoch``, ``round``, ``task``, ``job``.  Every key present
must match the injection point; a rule fires once per process unless ``repeat=1``.

Injection points call :func:`point` with their context, e.g.
``point("round", rank=r, epoch=e, round=i, task="train")``.
"""
from __future__ import annotations

import os
import time
from typing import Dict, List

_rules: List[Dict[str, str]] = []
_fired = set()
_loaded = False


def configure(spec: str):
    global _rules, _loaded
    _rules = []
    _fired.clear()
    for i, part in enumerate(x for x in (spec or "").split(";") if x.strip()):
        fields = part.strip().split(":")
        rule = {"action": fields[0], "_id": str(i)}
        for f in fields[1:]:
            if "=" in f:
                k, v = f.split("=", 1)
                rule[k.strip()] = v.strip()
        _rules.append(rule)
    _loaded = True


def _ensure():
    if not _loaded:
        configure(os.environ.get("KUBEML_FAULT", ""))


def point(where: str, **ctx):
    _ensure()
    if not _rules:
        return
    for r in _rules:
        if r.get("at", where) != where:
            continue
        ok = True
        for k in ("rank", "epoch", "round", "task", "job"):
            if k in r and str(ctx.get(k)) != r[k]:
                ok = False
                break
        if not ok:
            continue
        if r["_id"] in _fired and r.get("repeat") != "1":
            continue
        _fired.add(r["_id"])
        act = r["action"]
        if act == "kill":
            os._exit(17)
        if act == "raise":
            raise RuntimeError(f"injected fault at {where} {ctx}")
        if act == "hang":
            time.sleep(float(r.get("secs", "3600")))
