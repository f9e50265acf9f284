"""K-step model averaging (K-AVG / local SGD) — the reference's training algorithm.

Reference semantics:
* every worker trains on its shard for K local minibatch steps (K = -1: a whole epoch),
* then ALL model state (parameters and BN buffers, everything in ``state_dict``) is
  averaged over the workers that are still contributing (ml/pkg/model/model.go:249-302,
  parallelSGD.go:26-54; int64 buffers use integer division),
* each worker continues from the average and resets its optimizer state
  (python/kubeml/kubeml/network.py:121-128, 208-217).

MI355X-native (GPU workers): the model lives in ONE persistent fp32 ``state`` buffer
(nn/flat.py: master parameters | BN running stats | int64 counters as fp32 | count
slot).  A round is three launches on the compute stream and no host synchronisation:

    kavg_pack    int64 counters -> fp32 slots, count slot := participate
    all-reduce   SUM of the whole buffer (RCCL over xGMI)
    kavg_finish  x *= 1/count (divisor read on device), bf16 shadow refreshed in the
                 same pass, counters floored back to int64

On one node the all-reduce and the finish are ONE collective (``TorchComm.kavg_peer``, default
on GPU groups, ``KUBEML_KAVG_PEER=0`` keeps RCCL): the peer-memory two-shot over IPC-mapped
HBM (parallel/peer.py, comm.hip ``kml_peer_kavg``) reads 2 (P-1)/P of the state per rank over
xGMI and applies the average, the shadow refresh and the counter unpack in its reduce-scatter
and all-gather epilogues, so no extra pass over the 87 MB state follows the exchange.  The
transport passes a self-test that includes a fused round before it is used; on failure every
rank keeps the RCCL all-reduce + finish pair.

Workers that ran out of data (uneven ``split_minibatches``) send zeros and a zero
count, so the divisor is the number of contributing ranks, exactly like the
reference's partial merge rounds (ml/pkg/train/job.go:380-431).  CPU workers (gloo /
the in-process fake backend) run the same algorithm with torch ops.
"""
from __future__ import annotations

import time
from typing import List, Tuple

import torch

from .comm import Comm


class ModelAverager:
    def __init__(self, module: torch.nn.Module):
        self.module = module
        self.last_seconds = 0.0   # host time of the last average_ call (metrics)
        self.force = False        # run rounds on a 1-rank group too (single-GPU rehearsal)
        self.fused_rounds = 0     # rounds that ran as one fused peer-memory collective

    def _all_reduce(self, comm: Comm, t: torch.Tensor):
        if comm.world == 1 and self.force and hasattr(comm, "dist"):
            comm.dist.all_reduce(t, group=comm.group)      # 1-rank rehearsal: the collective runs
            return t
        return comm.all_reduce_(t)

    def _buffers(self) -> List[Tuple[str, torch.Tensor]]:
        return [(n, b) for n, b in self.module.named_buffers() if b is not None]

    def _space(self):
        sp = getattr(self.module, "_kml_flat", None)
        if sp is not None and getattr(sp, "state", None) is not None and sp.device.type == "cuda":
            return sp
        return None

    @torch.no_grad()
    def average_(self, comm: Comm, participate: bool = True) -> int:
        """Average the model over the group.  GPU: returns -1 (the participant count
        stays on the device); CPU: returns the participant count."""
        if comm.world == 1 and not (self.force and hasattr(comm, "dist")):
            return 1 if participate else 0
        t0 = time.perf_counter()
        sp = self._space()
        try:
            if sp is not None:
                return self._average_flat(comm, sp, participate)
            return self._average_host(comm, participate)
        finally:
            self.last_seconds = time.perf_counter() - t0

    def _average_flat(self, comm: Comm, sp, participate: bool) -> int:
        from ..ops import kernels as K
        arena = sp.i64_arena_now()
        if not participate:
            K.memset_(sp.state)
        K.kavg_pack_(sp.state, arena, sp.i64_off, sp.n_i64, sp.count_idx, participate)
        pk = comm.kavg_peer(sp.state) if hasattr(comm, "kavg_peer") and comm.world > 1 else None
        if pk is not None:
            # one fused round on the peer-memory two-shot (comm.hip kml_peer_kavg)
            pk.kavg_(sp.state, sp.count_idx, sp.numel, sp.shadow, arena, sp.i64_off,
                     sp.n_i64 if arena is not None else 0)
            self.fused_rounds += 1
        else:
            self._all_reduce(comm, sp.state)
            K.kavg_finish_(sp.state, sp.numel, sp.count_idx, sp.shadow, arena, sp.i64_off, sp.n_i64)
        self._average_other(comm, sp, participate)
        return -1

    def _average_other(self, comm: Comm, sp, participate: bool):
        """Buffers outside the fp32 state (other float dtypes, int32 / bool, non-scalar int64):
        one fp64 side pack + count, averaged like the reference's merger (integer buffers use
        floor division, parallelSGD.go:26-54)."""
        others = getattr(sp, "other_buffers", None)
        if not others:
            return
        ts = [getattr(m, n) for m, n in others]
        pack = torch.cat([t.detach().reshape(-1).double() for t in ts] +
                         [torch.ones(1, dtype=torch.float64, device=ts[0].device)])
        if not participate:
            pack.zero_()
        self._all_reduce(comm, pack)
        cnt = pack[-1:].clamp_min(1.0)
        off = 0
        with torch.no_grad():
            for t in ts:
                k = t.numel()
                v = pack[off:off + k].view(t.shape) / cnt
                if t.is_floating_point():
                    t.copy_(v.to(t.dtype))
                else:
                    t.copy_(torch.floor(v + 1e-9).to(t.dtype))
                off += k

    def _average_host(self, comm: Comm, participate: bool) -> int:
        """CPU path: pack everything into one fp32 vector (+count), one all-reduce."""
        bufs = self._buffers()
        params = [p for p in self.module.parameters()]
        pieces = [p.data.reshape(-1).float() for p in params] + [b.reshape(-1).float() for _, b in bufs]
        cnt = torch.tensor([1.0 if participate else 0.0])
        pack = torch.cat(pieces + [cnt]) if pieces else cnt
        if not participate:
            pack.zero_()
        self._all_reduce(comm, pack)
        n = int(round(float(pack[-1])))
        if n == 0:
            return 0
        pack[:-1].div_(n)
        off = 0
        for p in params:
            k = p.numel()
            p.data.copy_(pack[off:off + k].view_as(p.data))
            off += k
        for _, b in bufs:
            k = b.numel()
            v = pack[off:off + k].view_as(b)
            if b.is_floating_point():
                b.copy_(v)
            else:  # reference: integer layers use integer division (parallelSGD.go:26-54)
                b.copy_(torch.floor(v + 1e-3).to(b.dtype))
            off += k
        return n

    @torch.no_grad()
    def average_buffers_(self, comm: Comm):
        """Average only the module buffers (BN running statistics and counters) over the
        group.  Used by the synchronous gradient-all-reduce path, where parameters are
        identical on every rank by construction: BN running statistics follow a linear
        recurrence with rank-independent coefficients, so averaging them once at the end
        of an epoch equals averaging them after every step (K = 1 reference semantics)."""
        if comm.world == 1:
            return
        sp = self._space()
        if sp is not None:
            from ..ops import kernels as K
            arena = sp.i64_arena_now()
            seg = sp.state[sp.numel:]
            K.kavg_pack_(sp.state, arena, sp.i64_off, sp.n_i64, sp.count_idx, True)
            comm.all_reduce_(seg)
            # parameters are untouched: finish only over the buffer range (shadow not needed)
            K.kavg_finish_(seg, 0, sp.count_idx - sp.numel, None, arena, sp.i64_off - sp.numel, sp.n_i64)
            self._average_other(comm, sp, True)
            return
        bufs = self._buffers()
        if not bufs:
            return
        pack = torch.cat([b.reshape(-1).float() for _, b in bufs])
        comm.all_reduce_(pack)
        pack.div_(comm.world)
        off = 0
        for _, b in bufs:
            k = b.numel()
            v = pack[off:off + k].view_as(b)
            b.copy_(v if b.is_floating_point() else torch.floor(v + 1e-3).to(b.dtype))
            off += k

    @torch.no_grad()
    def broadcast_(self, comm: Comm, src: int = 0):
        """Make every worker hold rank ``src``'s model (init / elastic scale-up)."""
        if comm.world == 1:
            return
        sp = self._space()
        if sp is not None:
            comm.broadcast_(sp.state, src)     # parameters + buffers + counters slots
            for m, n in getattr(sp, "other_buffers", None) or ():
                t = getattr(m, n)
                c = t.contiguous()
                comm.broadcast_(c, src)
                if c.data_ptr() != t.data_ptr():
                    t.copy_(c)
            from ..ops import kernels as K
            arena = sp.i64_arena_now()
            if arena is not None:
                # counters travel as int64 too (their fp32 slots are only packed per round)
                comm.broadcast_(arena, src)
            sp.refresh_shadow()
            return
        sp = getattr(self.module, "_kml_flat", None)
        if sp is not None:
            comm.broadcast_(sp.master, src)
        else:
            for p in self.module.parameters():
                t = p.data.contiguous()
                comm.broadcast_(t, src)
                p.data.copy_(t)
        for _, b in self._buffers():
            t = b.contiguous()
            comm.broadcast_(t, src)
            b.copy_(t)
        if sp is not None:
            sp.refresh_shadow()


class AsyncModelAverager(ModelAverager):
    """Overlapped K-AVG with staleness 1 (opt-in, recorded in the history).

    The synchronous round (reference python/kubeml/kubeml/network.py:289-306) stops every
    worker until the average is back.  Here the all-reduce of round r is launched on the
    communicator's stream and the workers keep training round r+1 from their own model;
    at the end of round r+1 the average of round r replaces the stale base the local
    progress was made on:

        x_i  <-  mean_j x_j^(r)  +  (x_i^now - x_i^(r))

    and round r+1's all-reduce starts from the corrected model.  :meth:`flush_` applies the
    last pending average and then averages synchronously, so every worker ends the task with
    the same model (the reference's final merge).  Every rank must take part in every round
    (uneven tails go through :meth:`flush_` and the synchronous path).  Memory: two extra
    copies of the model state (the in-flight sum and the snapshot it was taken from).
    """

    def __init__(self, module: torch.nn.Module):
        super().__init__(module)
        self._pending = None      # (work | None, send, snap, tensors)
        self.rounds_overlapped = 0
        self._bufs = None         # (flat, snap) reused across rounds (flat-space GPU path)

    def _tensors(self):
        sp = self._space()
        if sp is not None:
            return [sp.state[:sp.i64_off]], sp
        return [p.data for p in self.module.parameters()] + [b for _, b in self._buffers() if b.is_floating_point()], None

    def _launch(self, comm: Comm, flat: torch.Tensor):
        """Async SUM of ``flat`` over the group; returns a waitable (None when the comm
        backend has no async collectives: the sum is then already done)."""
        dist_ = getattr(comm, "dist", None)
        if dist_ is not None and (comm.world > 1 or self.force):
            return dist_.all_reduce(flat, group=comm.group, async_op=True)
        self._all_reduce(comm, flat)
        return None

    @property
    def pending(self) -> bool:
        return self._pending is not None

    @torch.no_grad()
    def average_(self, comm: Comm, participate: bool = True) -> int:
        """One overlapped round.  Every rank must participate (callers route rounds in which
        some worker has no data through :meth:`flush_`, on every rank alike)."""
        if comm.world == 1 and not (self.force and hasattr(comm, "dist")):
            return 1 if participate else 0
        if not participate:
            raise ValueError("AsyncModelAverager.average_: every rank must participate (use flush_)")
        t0 = time.perf_counter()
        ts, sp = self._tensors()
        self._apply_pending(comm, ts, sp)
        if sp is not None and ts[0].is_cuda:
            # one fused pass (ops.kernels.kavg_snap_) into two round buffers kept across rounds
            x = ts[0]
            if self._bufs is None or self._bufs[0].numel() != x.numel():
                self._bufs = (torch.empty_like(x), torch.empty_like(x))
            flat, snap = self._bufs
            from ..ops import kernels as K
            K.kavg_snap_(x, flat, snap)
        else:
            flat = torch.cat([t.reshape(-1).float() for t in ts]) if len(ts) > 1 else ts[0].detach().clone()
            snap = flat.clone()
        work = self._launch(comm, flat)
        self._pending = (work, flat, snap)
        self.rounds_overlapped += 1
        self.last_seconds = time.perf_counter() - t0
        return -1

    def _apply_pending(self, comm: Comm, ts, sp):
        if self._pending is None:
            return
        work, flat, snap = self._pending
        self._pending = None
        if work is not None:
            work.wait()
        if sp is not None and ts[0].is_cuda and len(ts) == 1:
            # x <- x + (avg - snap) with the shadow refresh, one pass (same arithmetic order)
            from ..ops import kernels as K
            K.kavg_async_apply_(ts[0], flat, snap, sp.shadow, comm.world, sp.numel if sp.shadow is not None else 0)
            for p in sp.params:
                p._kml_shadow_version = p._version
            return
        # x <- avg + (x - snap), per tensor of the flat layout
        flat.div_(comm.world).sub_(snap)
        off = 0
        for t in ts:
            k = t.numel()
            t.add_(flat[off:off + k].view_as(t).to(t.dtype))
            off += k
        if sp is not None:
            sp.refresh_shadow()

    @torch.no_grad()
    def flush_(self, comm: Comm, participate: bool = True):
        """Apply the in-flight average, then one synchronous average (all ranks identical)."""
        if comm.world == 1 and not (self.force and hasattr(comm, "dist")):
            return
        ts, sp = self._tensors()
        self._apply_pending(comm, ts, sp)
        ModelAverager.average_(self, comm, participate)
