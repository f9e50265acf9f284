"""Communicator abstraction for the worker group of a job.

Backends
--------
* ``TorchComm``  — ``torch.distributed`` process group: ``nccl`` (= RCCL on ROCm,
  xGMI between the MI355X of one node) for GPU workers, ``gloo`` for CPU workers.
  Elastic parallelism uses sub-groups of the first P ranks, created once per P
  (every world rank must take part in ``new_group``) — the MI355X analogue of the
  reference re-invoking N serverless functions each epoch (ml/pkg/train/job.go:196-215).
* ``LocalComm``  — a single worker (world 1): every collective is the identity.
* ``ThreadComm`` — N ranks as threads of one process sharing memory; reductions go
  through the native ``kml_average_f32``/``kml_sum_f32`` merger.  This is the
  "fake comm backend" for testing K-AVG and elastic semantics without processes.

All collectives act on flat tensors (fp32 parameter/gradient buffers), never on
per-layer tensors: one collective per sync instead of the reference's per-layer
Redis round-trips (network.py:424-461, model.go:135-181).
"""
from __future__ import annotations

import os
import threading
from typing import Dict, List, Optional

import torch


class Comm:
    rank: int = 0
    world: int = 1

    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        raise NotImplementedError

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        raise NotImplementedError

    def barrier(self):
        raise NotImplementedError

    def all_gather_object(self, obj) -> list:
        raise NotImplementedError

    def check(self):
        """Raise if a collective of this group failed asynchronously (peer transport)."""

    # ------------------------------------------------------------------ helpers
    def average_(self, tensors: List[torch.Tensor], participate: bool = True) -> int:
        """Masked average: ranks with ``participate=False`` contribute zeros and are
        excluded from the divisor (reference: only functions still reporting are
        averaged, ml/pkg/train/job.go:380-431).  Returns the participant count."""
        dev = tensors[0].device
        cnt = torch.tensor([1.0 if participate else 0.0], dtype=torch.float32, device=dev)
        self.all_reduce_(cnt)
        n = int(round(float(cnt.item())))
        if n == 0:
            return 0
        for t in tensors:
            if not participate:
                t.zero_()
            self.all_reduce_(t)
            if t.is_floating_point():
                t.div_(n)
            else:
                t.copy_(torch.div(t, n, rounding_mode="floor"))
        return n

    def sub(self, parallelism: int) -> "Comm":
        """Communicator of ranks [0, parallelism) (elastic resize); self if equal."""
        if parallelism == self.world:
            return self
        raise NotImplementedError


class LocalComm(Comm):
    def __init__(self, device=None):
        self.rank, self.world = 0, 1

    def all_reduce_(self, t, op="sum"):
        return t

    def broadcast_(self, t, src=0):
        return t

    def barrier(self):
        pass

    def all_gather_object(self, obj):
        return [obj]

    def sub(self, parallelism):
        if parallelism != 1:
            raise ValueError("LocalComm has one rank")
        return self


_OPS = {"sum": "SUM", "max": "MAX", "min": "MIN", "avg": "AVG"}


class TorchComm(Comm):
    """torch.distributed group (RCCL over xGMI on MI355X, gloo on CPU).

    ``peer_data=True`` (GPU workers bootstrapped over gloo — e.g. several workers packed on one
    GPU, which RCCL refuses): the data plane is the peer-memory transport.  fp32 CUDA sums,
    averages and broadcasts go through a :class:`~kubeml_amd.parallel.peer.PeerAllReduce` grown
    on demand to the largest tensor seen (growing is collective; every member reduces the same
    sizes in the same order, so they grow together); other CUDA dtypes bounce through host
    memory over gloo."""

    def __init__(self, group=None, ranks: Optional[List[int]] = None, parent: "TorchComm" = None,
                 peer_data: bool = False):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.ranks = ranks if ranks is not None else list(range(dist.get_world_size()))
        grank = dist.get_rank()
        self.rank = self.ranks.index(grank) if grank in self.ranks else -1
        self.world = len(self.ranks)
        self._subs: Dict[int, "TorchComm"] = {}
        self._parent = parent
        self.peer_data = peer_data
        self.peer = None          # small/large fp32 reductions (enable_peer / peer_data)
        self.grad_peer = None     # the train step's gradient all-reduce (engine/dp.py, plan "peer")
        self.kavg_p = None        # fused K-AVG rounds over RCCL groups (kavg_peer)
        self._kavg_off = False    # its self-test failed: K-AVG stays on the RCCL all-reduce

    @property
    def member(self) -> bool:
        return self.rank >= 0

    def enable_peer(self, cap_bytes: Optional[int] = None):
        """Collective over this group: route fp32 sums/averages that fit ``cap_bytes`` per slot
        (default ``KUBEML_PEER_MB``, 8 MB) through the peer-memory all-reduce over xGMI
        (:mod:`kubeml_amd.parallel.peer`: one-shot for small, two-shot for large buffers)
        instead of RCCL.  GPU groups of one node only."""
        if self.world > 1 and self.peer is None:
            from .peer import DEFAULT_CAP, PeerAllReduce
            self.peer = PeerAllReduce(self.group, cap_bytes or DEFAULT_CAP)
        return self

    def check(self):
        """Raise :class:`~kubeml_amd.parallel.peer.PeerCommError` if a peer all-reduce of
        this group (or of its sub-groups) timed out; synchronises the device.  A poisoned
        transport is dropped first (its results are NaN for good): the next collective that
        needs one builds a fresh one, collectively."""
        err = None
        for name in ("peer", "grad_peer", "kavg_p"):
            p = getattr(self, name, None)
            if p is None:
                continue
            try:
                p.check()
            except Exception as e:
                err = err or e
                self._drop(name)
        for c in self._subs.values():
            try:
                c.check()
            except Exception as e:
                err = err or e
        if err is not None:
            raise err

    def _drop(self, name):
        """Unmap and free a transport WITHOUT a group barrier (its group may be broken)."""
        p = getattr(self, name, None)
        setattr(self, name, None)
        if p is not None:
            try:
                p._release()
            except Exception:
                pass

    def drop_peers(self):
        """Forget every peer transport of this group and its sub-groups (non-collective)."""
        for name in ("peer", "grad_peer", "kavg_p"):
            self._drop(name)
        for c in self._subs.values():
            c.drop_peers()

    def _peer_for(self, t, need_algo="auto"):
        """The peer transport for ``t`` (grown collectively when ``t`` no longer fits), or None."""
        if self.peer is not None and self.peer.supports(t):
            return self.peer
        if not (self.peer_data and t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
            return None
        from .peer import DEFAULT_CAP, PeerAllReduce, slot_bytes
        cap = max(DEFAULT_CAP, slot_bytes(t.numel(), self.world, "twoshot"), slot_bytes(t.numel(), self.world, "oneshot"))
        if self.peer is not None:
            cap = max(cap, self.peer.cap)
            self.peer.close()
        self.peer = PeerAllReduce(self.group, cap_bytes=cap, device=t.device)
        return self.peer

    def kavg_peer(self, t):
        """The peer transport for a fused K-AVG round over ``t`` (the flat fp32 state buffer):
        the two-shot with the average, shadow refresh and counter unpack in its epilogues
        (parallel/kavg.py), or None (all-reduce + ``kavg_finish_``).  peer_data groups use
        their data-plane transport; RCCL groups build one sized for the state on first use —
        collective: every member averages the same state in the same round — and keep it only
        if its self-test (which includes a fused round) passes on every rank.
        ``KUBEML_KAVG_PEER=0`` keeps RCCL."""
        if self.world == 1 or not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
            return None
        if self.peer_data:
            p = self._peer_for(t)
            return p if p is not None and p.supports_kavg(t) else None
        if getattr(self, "_kavg_off", False) or os.environ.get("KUBEML_KAVG_PEER", "1") == "0":
            return None
        if getattr(self, "kavg_p", None) is not None and self.kavg_p.supports_kavg(t):
            return self.kavg_p
        from .peer import slot_bytes, verified_peer
        if getattr(self, "kavg_p", None) is not None:
            self.kavg_p.close()
            self.kavg_p = None
        self.kavg_p = verified_peer(self.group, cap_bytes=slot_bytes(t.numel(), self.world, "twoshot"),
                                    device=t.device, kavg=True)
        self._kavg_off = self.kavg_p is None
        return self.kavg_p

    def _host_bounce(self, t, fn):
        """gloo collective on a host copy of a CUDA tensor (peer_data mode, non-fp32 dtypes)."""
        h = t.detach().cpu()
        fn(h)
        t.copy_(h)
        return t

    def all_reduce_(self, t, op="sum"):
        if self.world == 1:
            return t
        if op in ("sum", "avg"):
            peer = self._peer_for(t)
            if peer is not None:
                return peer.all_reduce_(t, 1.0 / self.world if op == "avg" else 1.0)
        o = getattr(self.dist.ReduceOp, _OPS[op])
        if self.peer_data and t.is_cuda:
            return self._host_bounce(t, lambda h: self.dist.all_reduce(h, op=o, group=self.group))
        self.dist.all_reduce(t, op=o, group=self.group)
        return t

    def broadcast_(self, t, src=0):
        if self.world == 1:
            return t
        if self.peer_data and t.is_cuda:
            peer = self._peer_for(t) if t.dtype == torch.float32 and t.is_contiguous() else None
            if peer is not None:
                # broadcast = sum with zeros from every other rank: exact (x + 0 = x)
                if self.rank != src:
                    t.zero_()
                return peer.all_reduce_(t, 1.0)
            return self._host_bounce(t, lambda h: self.dist.broadcast(h, src=self.ranks[src], group=self.group))
        self.dist.broadcast(t, src=self.ranks[src], group=self.group)
        return t

    def barrier(self):
        if self.world > 1:
            self.dist.barrier(group=self.group)

    def all_gather_object(self, obj):
        if self.world == 1:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj, group=self.group)
        return out

    def prepare_subgroups(self, max_p: Optional[int] = None):
        """Create the groups of ranks [0,p) for every p (collective over the world)."""
        max_p = max_p or self.world
        for p in range(1, max_p + 1):
            self.sub(p)

    def sub(self, parallelism):
        if parallelism == self.world:
            return self
        if not 1 <= parallelism <= self.world:
            raise ValueError(f"parallelism {parallelism} outside [1, {self.world}]")
        c = self._subs.get(parallelism)
        if c is None:
            ranks = self.ranks[:parallelism]
            g = self.dist.new_group(ranks=ranks)  # every world rank must call this, in order
            c = TorchComm(g, ranks, parent=self, peer_data=self.peer_data)
            self._subs[parallelism] = c
        return c


class _ThreadWorld:
    def __init__(self, n):
        self.n = n
        self.barrier = threading.Barrier(n)
        self.slots: List[Optional[torch.Tensor]] = [None] * n
        self.objs: List[object] = [None] * n
        self.result = None


class ThreadComm(Comm):
    """Ranks are threads of one process (tests / fake backend)."""

    def __init__(self, world: _ThreadWorld, rank: int, ranks: Optional[List[int]] = None):
        self._w = world
        self.ranks = ranks if ranks is not None else list(range(world.n))
        self.rank = rank
        self.world = len(self.ranks)
        self._subs: Dict[int, "ThreadComm"] = {}

    @staticmethod
    def create(n: int) -> List["ThreadComm"]:
        w = _ThreadWorld(n)
        return [ThreadComm(w, r) for r in range(n)]

    def _sync(self):
        self._w.barrier.wait()

    def all_reduce_(self, t, op="sum"):
        if self.world == 1:
            return t
        w = self._w
        w.slots[self.rank] = t
        self._sync()
        if self.rank == 0:
            srcs = [w.slots[i] for i in range(self.world)]
            acc = _native_reduce(srcs, op)
            w.result = acc
        self._sync()
        t.copy_(w.result)
        self._sync()
        return t

    def broadcast_(self, t, src=0):
        if self.world == 1:
            return t
        w = self._w
        if self.rank == src:
            w.result = t.clone()
        self._sync()
        t.copy_(w.result)
        self._sync()
        return t

    def barrier(self):
        if self.world > 1:
            self._sync()

    def all_gather_object(self, obj):
        w = self._w
        w.objs[self.rank] = obj
        self._sync()
        out = list(w.objs[: self.world])
        self._sync()
        return out

    def sub(self, parallelism):
        if parallelism == self.world:
            return self
        c = self._subs.get(parallelism)
        if c is None:
            c = ThreadComm(_shared_sub(self._w, parallelism), self.rank if self.rank < parallelism else -1,
                           list(range(parallelism)))
            self._subs[parallelism] = c
        return c


_SUBWORLDS: Dict[tuple, _ThreadWorld] = {}
_SUBLOCK = threading.Lock()


def _shared_sub(parent: _ThreadWorld, p: int) -> _ThreadWorld:
    with _SUBLOCK:
        key = (id(parent), p)
        w = _SUBWORLDS.get(key)
        if w is None:
            w = _ThreadWorld(p)
            _SUBWORLDS[key] = w
        return w


def _native_reduce(srcs: List[torch.Tensor], op: str) -> torch.Tensor:
    """Sum (or max/min) of same-shape CPU tensors through the native merger when possible."""
    if op == "sum" and all(s.dtype == torch.float32 and not s.is_cuda and s.is_contiguous() for s in srcs):
        try:
            from .. import _native
            out = torch.empty_like(srcs[0])
            import ctypes
            arr = (ctypes.c_void_p * len(srcs))(*[s.data_ptr() for s in srcs])
            rc = _native.RT.raw("kml_sum_f32", out.data_ptr(), arr, len(srcs), out.numel(), 4)
            if rc == 0:
                return out
        except Exception:
            pass
    acc = srcs[0].clone()
    for s in srcs[1:]:
        if op == "sum":
            acc += s
        elif op == "max":
            torch.maximum(acc, s, out=acc)
        elif op == "min":
            torch.minimum(acc, s, out=acc)
    return acc


def from_env(device=None) -> Comm:
    """Communicator for this process: the default torch.distributed group if
    initialised, else a LocalComm."""
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return TorchComm()
    except Exception:
        pass
    return LocalComm(device)
