"""How a data-parallel step moves its gradient.

A :class:`CommPlan` names the transport, the schedule and the wire precision of the per-step
gradient all-reduce:

* ``backend``  ``"peer"`` — the two-shot peer-memory all-reduce of :mod:`.peer` (plain
  kernels, captured in the step's hipGraph, bit-identical results on every rank), or
  ``"rccl"`` — RCCL over xGMI through ``torch.distributed``.
* ``schedule`` ``"end"`` — one all-reduce of the whole flat gradient after the backward, on
  the compute stream with the whole chip; ``"overlap"`` — one all-reduce per backward stage
  on a side stream while the next stage's backward runs; ``"shard"`` (peer only) — ZeRO-1:
  reduce-scatter of the fp32 gradient read in place from the peers, the optimizer on this
  rank's 1/P of the master (fused into the reduce for SGD), all-gather of the bf16 shadow
  (:class:`~kubeml_amd.parallel.peer.PeerShard`; the wire field is ignored: fp32 gradient,
  bf16 weights, which is what the forward computes with anyway); ``"shardov"`` — the same
  per backward stage on a side stream: each stage's reduce-scatter + SGD + all-gather runs as
  soon as its gradients are final, beside the backward of the stages before it (fused SGD,
  models with ``stages()``; otherwise it runs as ``"shard"``); ``"shardride"`` — the same per
  stage for the stages whose gradients are final early (``model.comm_ride_plan()``: ResNet's
  layer4 + fc, then layer3), but as rider blocks of later backward launches on the SAME queue
  (peer.ShardRider), so only the rest of the space is exchanged after the backward.
* ``wire``     fp32, or bf16 (half the link bytes; the sum accumulates in fp32).
* ``max_blocks`` the grid cap of every peer launch (the CUs the collective may hold).

Why the choice is measured, not assumed: the ResNet-34 backward is latency-bound (~100
dependent launches of 4-20 µs), and ANY kernel resident on a second queue slows each of its
dispatches by ~3 µs (``profiles/launch_fusion_r2.md``) — the overlapped schedule pays that
for the whole time its collective runs.  ``tools/interference_probe.py`` measures the step
with a side-queue streamer of an N=8 all-reduce's per-GPU bytes at several block caps, and the
one-GPU cost of each schedule; it writes ``kubeml_amd/parallel/comm_plan.json``, which
:func:`choose_plan` reads.  ``KUBEML_COMM_PLAN=backend:schedule:wire[:blocks]`` overrides it
(e.g. ``rccl:overlap:fp32``).

Reference counterpart: the TrainJob's per-round merge through RedisAI
(ml/pkg/train/job.go:368-442, ml/pkg/model/model.go:249-302).
"""
from __future__ import annotations

import json
import os
from dataclasses import asdict, dataclass
from typing import Optional

import torch

PLAN_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "comm_plan.json")
_WIRES = {"fp32": torch.float32, "bf16": torch.bfloat16}


@dataclass
class CommPlan:
    backend: str = "peer"          # "peer" | "rccl"
    schedule: str = "end"          # "end" | "overlap"
    wire: str = "fp32"             # "fp32" | "bf16"
    max_blocks: int = 256
    source: str = "default"

    def __post_init__(self):
        if self.backend not in ("peer", "rccl"):
            raise ValueError(f"backend must be peer or rccl, not {self.backend!r}")
        if self.schedule not in ("end", "overlap", "shard", "shardov", "shardride"):
            raise ValueError(f"schedule must be end, overlap, shard, shardov or shardride, not {self.schedule!r}")
        if self.schedule in ("shard", "shardov", "shardride") and self.backend != "peer":
            raise ValueError("the shard schedules run on the peer backend")
        if self.wire not in _WIRES:
            raise ValueError(f"wire must be fp32 or bf16, not {self.wire!r}")
        self.max_blocks = max(1, int(self.max_blocks))

    @property
    def wire_dtype(self) -> torch.dtype:
        return _WIRES[self.wire]

    def tag(self) -> str:
        t = f"{self.backend}:{self.schedule}:{self.wire}"
        return t + (f":{self.max_blocks}" if self.backend == "peer" else "")

    def to_dict(self) -> dict:
        return asdict(self)


def parse_plan(spec: str, source: str = "env") -> CommPlan:
    """``backend:schedule:wire[:max_blocks]`` -> CommPlan."""
    parts = [p.strip() for p in spec.split(":") if p.strip()]
    if not 3 <= len(parts) <= 4:
        raise ValueError(f"comm plan {spec!r}: expected backend:schedule:wire[:max_blocks]")
    return CommPlan(parts[0], parts[1], parts[2], int(parts[3]) if len(parts) == 4 else 256, source)


def load_table(path: str = PLAN_FILE) -> Optional[dict]:
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def choose_plan(world: int, grad_bytes: int, *, override: Optional[str] = None, table: Optional[dict] = None,
                gpu: bool = True) -> CommPlan:
    """The plan for a ``world``-rank step over a ``grad_bytes`` fp32 gradient.

    Precedence: ``override`` / ``KUBEML_COMM_PLAN`` > the measured table's choice for the
    nearest world size > the default (peer, end of step, fp32 — exact, no side-queue
    interference).  CPU groups always use the torch backend (gloo)."""
    spec = override or os.environ.get("KUBEML_COMM_PLAN")
    if spec:
        return parse_plan(spec, "override" if override else "env")
    if not gpu:
        return CommPlan("rccl", "overlap", "fp32", source="cpu (gloo)")
    table = table if table is not None else load_table()
    if table and table.get("choice"):
        ch = table["choice"]
        key = str(world) if str(world) in ch else (min(ch, key=lambda k: abs(int(k) - world)) if ch else None)
        if key is not None:
            return parse_plan(ch[key], f"{os.path.basename(PLAN_FILE)} (world {key})")
    return CommPlan(source="default")
