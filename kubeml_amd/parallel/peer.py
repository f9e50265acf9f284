"""Peer-memory all-reduce over IPC-mapped HBM on one xGMI-connected node.

On an MI355X node every GPU reaches every peer's HBM over its own xGMI link, so a collective
can be a handful of ordinary kernels that read the peers' bytes directly — no ring, no proxy
thread, nothing outside the stream (``csrc/kernels/comm.hip``):

* **one-shot** (small buffers: LeNet's parameters, BN statistics, loss / count scalars): one
  barrier, then every rank reads all P inputs and sums them — latency-optimal.
* **two-shot** (large buffers: the flat gradient of a ResNet-34 step): reduce-scatter, then
  all-gather — each rank reads 2(P-1)/P of the buffer over its 7 links, the ring optimum,
  with two barriers instead of the ring's 2(P-1) steps.  ``wire=torch.bfloat16`` rounds the
  slots to bf16 (half the link bytes; sums accumulate in fp32).

Both are stream-ordered launches whose state (barrier sequence, call parity) lives on the
device, so they capture into a hipGraph and replay; every rank ends with bit-identical
results (chunk q is reduced once, by rank q, in rank order).  ``max_blocks`` caps every
launch's grid: the whole chip at the end of a step, a few CUs beside a running backward.

Failure is loud.  A barrier wait is bounded by wall time (``KUBEML_PEER_TIMEOUT_S``, default
60 s); on expiry the call writes NaN and the group is poisoned — every later call writes NaN
at once — and :meth:`check` raises :class:`PeerCommError` (a ``MergeError``, the reference's
merge-failure error, ml/pkg/train/api.go:120-123).  Workers call :meth:`check` at every
K-AVG round and task end.

Regions are exchanged once, at construction, through the job's process group
(``all_gather_object`` of the IPC handles): construction is collective over the group.

Reference counterpart: the Go merger's sum of the per-function weights pulled from RedisAI
(ml/pkg/model/model.go:249-302) and the ParallelSGD average (ml/pkg/model/parallelSGD.go:26-54).
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional

import torch

from .._native import HIP
from ..api.errors import MergeError

DEFAULT_CAP = int(float(os.environ.get("KUBEML_PEER_MB", "8")) * 2**20)
ONESHOT_MAX_BYTES = 512 * 1024    # one-shot (latency-optimal) up to here, two-shot above
DEFAULT_TIMEOUT_S = float(os.environ.get("KUBEML_PEER_TIMEOUT_S", "60"))
ALGOS = {"oneshot": 0, "twoshot": 1}


class PeerCommError(MergeError):
    def __init__(self, message: str):
        super().__init__(message)


def slot_bytes(n: int, world: int, algo: str, wire=torch.float32) -> int:
    """Slot bytes one call of ``n`` fp32 elements needs (the region holds two slots)."""
    ve = 8 if wire == torch.bfloat16 else 4
    nvec = -(-n // ve)
    if algo == "twoshot":
        nvec = -(-nvec // world) * world
    return nvec * 16


class PeerAllReduce:
    """Collective over ``group`` (a torch.distributed group, or None for the world)."""

    MAX_RANKS = 8

    def __init__(self, group=None, cap_bytes: int = DEFAULT_CAP, device: Optional[torch.device] = None,
                 timeout_s: float = DEFAULT_TIMEOUT_S):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if self.world > self.MAX_RANKS:
            raise ValueError(f"peer all-reduce supports up to {self.MAX_RANKS} ranks (one node)")
        self.cap = (int(cap_bytes) + 15) // 16 * 16
        self.timeout_s = float(timeout_s)
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        with torch.cuda.device(self.device):
            region, ctrl = ctypes.c_void_p(), ctypes.c_void_p()
            HIP.call("kml_peer_alloc", "l p p", self.cap, ctypes.addressof(region), ctypes.addressof(ctrl))
            self.region, self.ctrl = region.value, ctrl.value
            nb = HIP.raw("kml_ipc_handle_bytes")
            h = (ctypes.c_char * nb)()
            HIP.call("kml_ipc_get_handle", "p p", self.region, ctypes.addressof(h))
            handles: List[bytes] = [b""] * self.world
            dist.all_gather_object(handles, bytes(h), group=group)
            self.opened: List[int] = []
            ptrs, err = [], ""
            try:
                for p, hb in enumerate(handles):
                    if p == self.rank:
                        ptrs.append(self.region)
                        continue
                    buf = (ctypes.c_char * nb).from_buffer_copy(hb)
                    out = ctypes.c_void_p()
                    HIP.call("kml_ipc_open", "p p", ctypes.addressof(buf), ctypes.addressof(out))
                    self.opened.append(out.value)
                    ptrs.append(out.value)
                torch.cuda.synchronize(self.device)
            except Exception as e:   # a rank that cannot map a peer must not leave the others waiting
                err = f"rank {self.rank}: {e!r}"[:300]
            self._regions = (ctypes.c_void_p * self.world)(*(ptrs + [0] * (self.world - len(ptrs))))
        errs: List[str] = [""] * self.world
        dist.all_gather_object(errs, err, group=group)   # every rank has mapped every region (or not)
        if any(errs):
            self._release()
            raise PeerCommError("peer all-reduce setup failed: " + "; ".join(e for e in errs if e))

    # ------------------------------------------------------------------ calls
    def pick_algo(self, t: torch.Tensor) -> str:
        return "oneshot" if t.numel() * 4 <= ONESHOT_MAX_BYTES or self.world == 1 else "twoshot"

    def supports(self, t: torch.Tensor, algo: str = "auto", wire=torch.float32) -> bool:
        if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.device == self.device):
            return False
        algo = self.pick_algo(t) if algo == "auto" else algo
        return slot_bytes(t.numel(), self.world, algo, wire) <= self.cap

    def all_reduce_(self, t: torch.Tensor, scale: float = 1.0, algo: str = "auto", wire=torch.float32,
                    max_blocks: Optional[int] = None) -> torch.Tensor:
        """t := scale * sum over ranks of t (in place; every rank, same order; capturable)."""
        if self.region is None:
            raise PeerCommError("peer all-reduce used after close()")
        algo = self.pick_algo(t) if algo == "auto" else algo
        if algo not in ALGOS:
            raise ValueError(f"algo must be one of {sorted(ALGOS)} or 'auto'")
        if wire not in (torch.float32, torch.bfloat16):
            raise ValueError("wire must be torch.float32 or torch.bfloat16")
        if not self.supports(t, algo, wire):
            raise ValueError(f"peer all-reduce: contiguous fp32 tensor on {self.device} needing at most "
                             f"{self.cap} slot bytes (got {t.numel()} elements, {t.dtype}, {t.device})")
        HIP.call("kml_peer_allreduce", "p p p p p i i l l f i i i d s", t.data_ptr(), t.data_ptr(),
                 ctypes.addressof(self._regions), self.region, self.ctrl, self.rank, self.world, self.cap,
                 t.numel(), float(scale), ALGOS[algo], int(wire == torch.bfloat16), int(max_blocks or 256),
                 self.timeout_s, torch.cuda.current_stream(self.device).cuda_stream)
        return t

    def supports_kavg(self, state: torch.Tensor) -> bool:
        return self.supports(state, "twoshot", torch.float32)

    def kavg_(self, state: torch.Tensor, count_idx: int, n_params: int = 0, shadow: Optional[torch.Tensor] = None,
              i64: Optional[torch.Tensor] = None, i64_off: int = 0, n_i64: int = 0,
              max_blocks: Optional[int] = None) -> torch.Tensor:
        """One K-AVG round in place on the flat state buffer (after ``kavg_pack_``): the
        two-shot sum with the average by the on-device count, the bf16 shadow refresh of
        ``[0, n_params)`` and the int64 counter unpack in its epilogues (comm.hip
        ``kml_peer_kavg``) — what ``all_reduce_`` + ``kavg_finish_`` do in two passes more."""
        if self.region is None:
            raise PeerCommError("peer all-reduce used after close()")
        if not self.supports_kavg(state):
            raise ValueError(f"peer K-AVG: contiguous fp32 state on {self.device} within {self.cap} slot bytes")
        if shadow is not None and (shadow.dtype != torch.bfloat16 or shadow.numel() < n_params):
            raise ValueError("peer K-AVG: shadow must be bf16 with n_params elements")
        if n_i64 and (i64 is None or i64.dtype != torch.int64 or i64.numel() < n_i64):
            raise ValueError("peer K-AVG: i64 arena must hold n_i64 int64 counters")
        HIP.call("kml_peer_kavg", "p p p p i i l l l l p p l i i d s", state.data_ptr(),
                 ctypes.addressof(self._regions), self.region, self.ctrl, self.rank, self.world, self.cap,
                 state.numel(), int(count_idx), int(n_params), 0 if shadow is None else shadow.data_ptr(),
                 0 if i64 is None else i64.data_ptr(), int(i64_off), int(n_i64), int(max_blocks or 256),
                 self.timeout_s, torch.cuda.current_stream(self.device).cuda_stream)
        return state

    def _kavg_self_test(self) -> bool:
        """Fused K-AVG round on a synthetic layout (integer patterns, one non-participating rank
        when world > 2) against the closed form computed with the same fp32 operations."""
        n = min(1 << 20, self.cap // 4 - 64)
        n -= n % 4
        if n < self.world * 64:
            return True
        count_idx, n_params, i64_off, n_i64 = n - 3, n - 67, n - 67, 40
        idx = torch.arange(n, device=self.device)
        base = (idx % 8).float()
        part = [r for r in range(self.world) if not (self.world > 2 and r == self.world - 1)]
        ok = True
        for _ in range(3):                      # both slot parities, then one more
            st = base * float(self.rank + 1) if self.rank in part else torch.zeros_like(base)
            st[count_idx] = 1.0 if self.rank in part else 0.0
            shadow = torch.empty(n_params, dtype=torch.bfloat16, device=self.device)
            arena = torch.empty(n_i64, dtype=torch.int64, device=self.device)
            self.kavg_(st, count_idx, n_params, shadow, arena, i64_off, n_i64)
            tot = base * float(sum(r + 1 for r in part))
            want = tot.clone()
            inv = torch.tensor(1.0, device=self.device) / float(max(len(part), 1))
            want[:count_idx] = tot[:count_idx] * inv
            want[count_idx] = float(len(part))
            ok = ok and bool(torch.equal(st, want)) and bool(torch.equal(shadow, want[:n_params].to(torch.bfloat16)))
            ok = ok and bool(torch.equal(arena, torch.floor(want[i64_off:i64_off + n_i64] + 1e-3).long()))
        return ok

    # ------------------------------------------------------------------ health
    def errors(self) -> int:
        """Timed-out barrier waits so far (non-zero: the group is poisoned, outputs are NaN)."""
        if self.ctrl is None:
            return 0
        out = ctypes.c_uint(0)
        HIP.call("kml_peer_errors", "p p", self.ctrl, ctypes.addressof(out))
        return int(out.value)

    def check(self):
        """Raise :class:`PeerCommError` if any wait of this group ever timed out (synchronises)."""
        n = self.errors()
        if n:
            raise PeerCommError(f"peer all-reduce: {n} barrier wait(s) on rank {self.rank}/{self.world} timed out "
                                f"after {self.timeout_s:g} s (a peer stopped calling); results since then are NaN")

    def self_test(self, n: Optional[int] = None, kavg: bool = False) -> bool:
        """Collective: run both algorithms and both wires on rank-dependent integer patterns
        (exact in bf16 and fp32) and compare with the closed-form sums; ``kavg``: also a fused
        K-AVG round (kml_peer_kavg), only for a transport that will run those — a K-AVG-only
        failure must not drop the gradient all-reduce to RCCL.  True on every rank only if every
        rank got exact results and no wait timed out."""
        ok = True
        try:
            big = min(n or 4 << 20, self.cap // 4 - 64)
            for numel, algo in ((4099, "oneshot"), (big, "twoshot")):
                if numel < self.world * 8:
                    continue
                idx = torch.arange(numel, device=self.device)
                base = (idx % 8).float()
                want = base * float(self.world * (self.world + 1) // 2)
                for wire in (torch.float32, torch.bfloat16):
                    if not self.supports(base, algo, wire):
                        continue
                    for _ in range(3):          # both slot parities, then one more
                        t = base * float(self.rank + 1)
                        self.all_reduce_(t, 1.0, algo=algo, wire=wire)
                        ok = ok and bool(torch.equal(t, want))
            if kavg:
                kok = self._kavg_self_test()
                if not kok:
                    import logging
                    logging.getLogger("kubeml.peer").warning("rank %d: fused K-AVG round failed its self-test",
                                                             self.rank)
                ok = kok and ok
            torch.cuda.synchronize(self.device)
            ok = ok and self.errors() == 0
            from ..utils import fault
            fault.point("shard_selftest", rank=self.rank)    # failure-path tests: this rank's check fails
        except Exception:
            ok = False
        flags: List[bool] = [False] * self.world
        self.dist.all_gather_object(flags, ok, group=self.group)
        return all(flags)

    def _release(self):
        for p in self.opened:
            try:
                HIP.call("kml_ipc_close", "p", p)
            except Exception:
                pass
        self.opened = []
        if self.region is not None:
            HIP.call("kml_peer_free", "p p", self.region, self.ctrl)
        self.region = self.ctrl = None

    def close(self):
        """Collective: unmap the peers' regions after everyone is done, then free our own."""
        if self.region is None:
            return
        torch.cuda.synchronize(self.device)
        self.dist.barrier(group=self.group)
        for p in self.opened:
            HIP.call("kml_ipc_close", "p", p)
        self.opened = []
        self.dist.barrier(group=self.group)
        HIP.call("kml_peer_free", "p p", self.region, self.ctrl)
        self.region = self.ctrl = None


def verified_peer(group=None, cap_bytes: int = DEFAULT_CAP, device: Optional[torch.device] = None,
                  log=None, kavg: bool = False) -> Optional["PeerAllReduce"]:
    """Collective: a :class:`PeerAllReduce` that passed :meth:`PeerAllReduce.self_test` on every
    rank, or None (every rank agrees) — callers then keep RCCL.  ``kavg``: the transport will run
    fused K-AVG rounds, so the test includes one.  ``KUBEML_PEER_SELFTEST=0`` skips the test."""
    try:
        p = PeerAllReduce(group, cap_bytes=cap_bytes, device=device)
    except PeerCommError as e:
        if log:
            log(f"peer all-reduce unavailable, using RCCL: {e}")
        return None
    if os.environ.get("KUBEML_PEER_SELFTEST", "1") == "0" or p.self_test(kavg=kavg):
        return p
    if log:
        log("peer all-reduce failed its self-test on this node, using RCCL")
    try:
        p.close()
    except Exception:
        pass
    return None


# ---------------------------------------------------------------------------------------------
# IPC-exportable device buffers and the sharded (ZeRO-1) update
# ---------------------------------------------------------------------------------------------
class _IpcBlock:
    """One hipMalloc allocation (an IPC handle covers it from its base) exposed to torch through
    ``__cuda_array_interface__``; freed when the last tensor viewing it dies."""

    def __init__(self, nbytes: int, device: torch.device):
        out = ctypes.c_void_p()
        with torch.cuda.device(device):
            HIP.call("kml_ipc_alloc", "l p", int(nbytes), ctypes.addressof(out))
        self.ptr, self.nbytes, self.device = out.value, int(nbytes), device
        self.__cuda_array_interface__ = {"shape": (self.nbytes,), "typestr": "|u1", "data": (self.ptr, False),
                                         "version": 2}

    def __del__(self):
        try:
            if self.ptr:
                HIP.raw("kml_ipc_free", self.ptr)
        except Exception:
            pass
        self.ptr = None


_IPC_OK = None


def ipc_zeros(numel: int, dtype: torch.dtype, device) -> Optional[torch.Tensor]:
    """Zeroed device tensor at the base of its own hipMalloc allocation (so peers can map it with
    an IPC handle), or None where this torch build cannot wrap foreign device memory."""
    global _IPC_OK
    if _IPC_OK is False:
        return None
    device = torch.device(device)
    esz = torch.tensor([], dtype=dtype).element_size()
    try:
        blk = _IpcBlock(max(16, numel * esz), device)
        t = torch.as_tensor(blk, device=device)
        if t.data_ptr() != blk.ptr or t.device != device:
            raise RuntimeError("foreign device memory not wrapped in place")
        _IPC_OK = True
        return t[:numel * esz].view(dtype)
    except Exception as e:   # pragma: no cover - depends on the torch build
        if _IPC_OK is None:
            import logging
            logging.getLogger("kubeml.peer").warning("IPC flat buffers unavailable (%r): the sharded "
                                                     "update falls back to the all-reduce plans", e)
        _IPC_OK = False
        return None


def _device_ident(device) -> tuple:
    """Identity of the physical GPU behind ``device`` (PCI location), comparable across processes."""
    import socket
    props = torch.cuda.get_device_properties(device)
    pci = tuple(getattr(props, k, None) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
    if all(v is None for v in pci):
        pci = (torch.device(device).index, os.environ.get("HIP_VISIBLE_DEVICES"), os.environ.get("ROCR_VISIBLE_DEVICES"))
    return (socket.gethostname(),) + pci


def _handle_of(ptr: int) -> bytes:
    nb = HIP.raw("kml_ipc_handle_bytes")
    h = (ctypes.c_char * nb)()
    HIP.call("kml_ipc_get_handle", "p p", ptr, ctypes.addressof(h))
    return bytes(h)


class PeerShard:
    """ZeRO-1 data-parallel update of one flat parameter space over a one-node group.

    Every rank's fp32 gradient, fp32 master (the head of ``space.state``) and bf16 shadow are
    IPC buffers (:func:`ipc_zeros`); every rank maps every peer's.  One step is two launches
    (``csrc/kernels/comm.hip`` k_zs_rs / k_zs_gather): rank r reduces chunk r of the P gradients
    in rank order straight from the peers' HBM (fp32, exact sums, no staging copy) and applies
    the optimizer to its 1/P of the master — fused into the same pass for SGD — then every rank
    gathers the peers' freshly written bf16 shadow chunks, which are the weights the next forward
    reads.  The fp32 master is complete only on its owner's chunk; :meth:`gather_master` (one
    launch) completes it where the full master is read: K-AVG rounds, checkpoints, epoch ends.

    Link bytes per rank and step: 4(P-1)/P n + 2(P-1)/P n — an fp32-exact gradient at 3/4 of an
    fp32 all-reduce, with 1/P of the optimizer pass instead of all of it on every rank.
    Construction is collective over ``group``; failures are loud like :class:`PeerAllReduce`.
    Reference counterpart: the job's fp32 merge + average (ml/pkg/model/parallelSGD.go:26-54)."""

    def __init__(self, space, group=None, timeout_s: float = DEFAULT_TIMEOUT_S):
        import torch.distributed as dist
        self.dist, self.group, self.space = dist, group, space
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if self.world > PeerAllReduce.MAX_RANKS:
            raise ValueError(f"sharded update supports up to {PeerAllReduce.MAX_RANKS} ranks (one node)")
        # whether this rank's flat buffers are IPC-exportable is agreed collectively below: a
        # rank that bailed out here alone would leave its peers blocked in all_gather_object
        ipc_ok = bool(getattr(space, "ipc", False))
        self.timeout_s = float(timeout_s)
        self.device = space.device
        self.n = int(space.numel)
        self.chunk = -(-self.n // (self.world * 64)) * 64
        self.lo = min(self.n, self.rank * self.chunk)
        self.hi = min(self.n, self.lo + self.chunk)
        # ownership layout: segments (s0, s1, chunk); rank r owns [s0 + r chunk, s0 + (r+1) chunk)
        # of each.  One segment = the whole space; set_stages() cuts it per backward stage
        self.segments = [(0, self.n, self.chunk)]
        self._seg_ptrs: List[tuple] = []
        self.opened: List[int] = []
        self.region = self.ctrl = None
        err = ""
        with torch.cuda.device(self.device):
            hs = None
            if ipc_ok:
                region, ctrl = ctypes.c_void_p(), ctypes.c_void_p()
                HIP.call("kml_peer_alloc", "l p p", 16, ctypes.addressof(region), ctypes.addressof(ctrl))
                self.region, self.ctrl = region.value, ctrl.value
                mine = [self.region, space.grad.data_ptr(), space.shadow.data_ptr(), space.state.data_ptr()]
                hs = [_handle_of(p) for p in mine]
            allh: List[list] = [None] * self.world
            dist.all_gather_object(allh, (hs, _device_ident(self.device)), group=group)
            if any(a[0] is None for a in allh):
                self._release()
                bad = [r for r, a in enumerate(allh) if a[0] is None]
                raise PeerCommError(f"sharded update needs IPC flat buffers on every rank (nn/flat.py); "
                                    f"ranks {bad} have none")
            # the barrier is a one-block launch of its own and the work kernels behind it never
            # spin (split): they run at full grid like any streaming kernel, with no per-block
            # fence, and ranks that share one GPU (packed workers, tests) cannot fill the CUs a
            # peer still needs to reach the barrier
            self.packed = len({a[1] for a in allh}) < self.world
            self.ranks_per_device = sum(1 for a in allh if a[1] == _device_ident(self.device))
            self.split = True
            allh = [a[0] for a in allh]
            cols: List[list] = [[0] * self.world for _ in range(4)]
            try:
                for p in range(self.world):
                    for k in range(4):
                        if p == self.rank:
                            cols[k][p] = mine[k]
                            continue
                        nb = len(allh[p][k])
                        buf = (ctypes.c_char * nb).from_buffer_copy(allh[p][k])
                        out = ctypes.c_void_p()
                        HIP.call("kml_ipc_open", "p p", ctypes.addressof(buf), ctypes.addressof(out))
                        self.opened.append(out.value)
                        cols[k][p] = out.value
                torch.cuda.synchronize(self.device)
            except Exception as e:
                err = f"rank {self.rank}: {e!r}"[:300]
            arr = ctypes.c_void_p * self.world
            self._flags, self._grads, self._shadows, self._states = (arr(*c) for c in cols)
        errs: List[str] = [""] * self.world
        dist.all_gather_object(errs, err, group=group)
        if any(errs):
            self._release()
            raise PeerCommError("sharded update setup failed: " + "; ".join(e for e in errs if e))
        space.master_sync = self.gather_master

    # ------------------------------------------------------------------ the step
    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def reduce_scatter(self, optimizer=None, advance=None, max_blocks: int = 256, stamp: Optional[int] = None):
        """Chunk ``[lo, hi)`` := sum over ranks.  With a fused-SGD ``optimizer`` the sum is
        applied at once (master, momentum, shadow of the chunk; 1/P folded in); else it lands in
        the own gradient chunk for :meth:`update_range`.  ``stamp``: device address of an int64 the
        barrier launch stamps (100 MHz wall clock) when timing the step's collectives."""
        if len(self.segments) != 1:
            raise PeerCommError("staged layout: use stage_step()")
        self._rs_call(self.lo, self.hi, optimizer, advance, max_blocks, stamp, clear_first=True)

    def _rs_call(self, lo, hi, optimizer, advance, max_blocks, stamp, clear_first=True):
        sp = self.space
        if self.region is None:
            raise PeerCommError("sharded update used after close()")
        fused = optimizer is not None
        mom = first = lr = None
        wd = momentum = dampening = 0.0
        nesterov = 0
        if fused:
            g = optimizer.param_groups[0]
            wd, momentum, dampening, nesterov = g["weight_decay"], g["momentum"], g["dampening"], int(g["nesterov"])
            lr = optimizer.lr_tensor(sp.device)
            if momentum != 0:
                mom = optimizer._bufs(sp, ["momentum"])["momentum"]
                first = optimizer.first_tensor(sp.device)
        ctr, ab, an = advance if advance is not None else (None, 0.0, 0.0)
        HIP.call("kml_zs_reduce_scatter", "p p p p i i l l i p p p p f f f i p f p f f i d i p s",
                 ctypes.addressof(self._flags), ctypes.addressof(self._grads), self.region, self.ctrl, self.rank,
                 self.world, int(lo), int(hi), int(fused), sp.master.data_ptr() if fused else None,
                 mom.data_ptr() if mom is not None else None, sp.shadow.data_ptr() if fused else None,
                 lr.data_ptr() if lr is not None else None, float(wd), float(momentum), float(dampening), nesterov,
                 first.data_ptr() if first is not None else None, 1.0 / self.world,
                 ctr.data_ptr() if ctr is not None else None, float(ab), float(an), int(max_blocks),
                 self.timeout_s, int(self.split), stamp, self._stream())
        if first is not None and clear_first:
            from ..ops import kernels as K
            K.fill_(first, 0.0)

    def all_gather_shadow(self, max_blocks: int = 256, stamp: Optional[int] = None):
        """Every rank's shadow := the owners' freshly updated chunks (closes the step's call;
        ``stamp``: its last block stamps the collective's end)."""
        HIP.call("kml_zs_all_gather", "p p p p i i l l i i i i d i p s", ctypes.addressof(self._flags),
                 ctypes.addressof(self._shadows), self.region, self.ctrl, self.rank, self.world, self.n,
                 self.chunk, 2, 2, 2, int(max_blocks), self.timeout_s, int(self.split), stamp, self._stream())
        self.space._master_stale = True

    # ------------------------------------------------------------------ staged layout
    def set_stages(self, ranges):
        """Cut the ownership per backward stage: ``ranges`` = contiguous flat ranges tiling the
        space; rank r then owns chunk r of EVERY range, so each stage's gradient can be
        reduce-scattered, applied and all-gathered on its own (:meth:`stage_step`) while the
        backward of the stages before it still runs.  Collective in effect (every rank must
        pass the same ranges); the master must be complete (sync_master) before the switch."""
        segs = []
        for s0, s1 in ranges:
            s0, s1 = int(s0), int(s1)
            if s1 <= s0:
                continue
            if s0 % 8 or (s1 % 8 and s1 != self.n):
                raise ValueError("stage ranges must start at multiples of 8 elements")
            segs.append((s0, s1, -(-(s1 - s0) // (self.world * 64)) * 64))
        if not segs or segs[0][0] != 0 or segs[-1][1] != self.n or any(a[1] != b[0] for a, b in zip(segs, segs[1:])):
            raise ValueError("stage ranges must tile the flat space in order")
        self.segments = segs
        arr = ctypes.c_void_p * self.world
        self._seg_ptrs = []
        for s0, s1, ch in segs:
            sh = arr(*[int(v) + 2 * s0 for v in self._shadows])
            st = arr(*[int(v) + 4 * s0 for v in self._states])
            self._seg_ptrs.append((sh, st))

    def owned(self):
        """[(lo, hi)] flat ranges whose master / optimizer state this rank keeps current."""
        out = []
        for s0, s1, ch in self.segments:
            lo = min(s1, s0 + self.rank * ch)
            out.append((lo, min(s1, lo + ch)))
        return out

    def stage_step(self, k: int, optimizer, advance=None, max_blocks: int = 256, first_stage: bool = True,
                   last_stage: bool = True, stamps=None):
        """Segment k of a staged layout: reduce-scatter + fused SGD on this rank's chunk of the
        segment, then the bf16 shadow all-gather of the segment.  ``first_stage`` /
        ``last_stage``: the first call of a step stamps the start, the last clears SGD's
        first-step flag, advances the data counter and stamps the end."""
        s0, s1, ch = self.segments[k]
        lo = min(s1, s0 + self.rank * ch)
        hi = min(s1, lo + ch)
        self._rs_call(lo, hi, optimizer, advance if last_stage else None, max_blocks,
                      stamps[0] if (stamps is not None and first_stage) else None, clear_first=last_stage)
        sh, _ = self._seg_ptrs[k]
        HIP.call("kml_zs_all_gather", "p p p p i i l l i i i i d i p s", ctypes.addressof(self._flags),
                 ctypes.addressof(sh), self.region, self.ctrl, self.rank, self.world, s1 - s0, ch, 2, 2, 2,
                 int(max_blocks), self.timeout_s, int(self.split),
                 stamps[1] if (stamps is not None and last_stage) else None, self._stream())
        self.space._master_stale = True

    # ------------------------------------------------------------------ rider slices
    # Progress offsets of the step's rider phases (kml_sgd.h KmlZsRider): stage s (0 or 1) of a
    # staged layout publishes READY = 2 s + 1 and DONE = 2 s + 2; the last AG phase advances the
    # base by 4 for the next step.  ctrl words 5..7 count the finished blocks of RS-0, RS-1, AG-1.
    RIDER_STAGES = 2

    def rider_slices(self, seg: int, kind: str, n_hosts: int, optimizer, blocks: int = 256) -> List["ShardRider"]:
        """The ``n_hosts`` slices of stage ``seg``'s reduce-scatter (``kind`` "rs": this rank's
        chunk, summed over every rank's gradient, fused SGD, shadow chunk published) or all-gather
        ("ag": the peers' shadow chunks) as riders (:class:`ShardRider`) for ``n_hosts`` later
        backward launches — every rank must build the same slices (same hosts, same blocks)."""
        if seg >= self.RIDER_STAGES or len(self.segments) <= seg:
            raise ValueError("rider slices need a staged layout (set_stages) and stage 0 or 1")
        if n_hosts < 1 or blocks < 1:
            raise ValueError("rider slices: at least one host launch and one block")
        sp = self.space
        s0, s1, ch = self.segments[seg]
        arr = ctypes.c_void_p * self.world
        if kind == "rs":
            lo = min(s1, s0 + self.rank * ch)
            hi = min(s1, lo + ch)
            if (hi - lo) % 4:
                raise ValueError("rider RS: the own chunk must hold whole fp32x4 vectors")
            a, b, nv = lo - s0, hi - s0, (hi - lo) // 4
            data = arr(*[int(v) + 4 * s0 for v in self._grads])
            g = optimizer.param_groups[0]
            lr = optimizer.lr_tensor(sp.device)
            mom = first = None
            if g["momentum"] != 0:
                mom = optimizer._bufs(sp, ["momentum"])["momentum"]
                first = optimizer.first_tensor(sp.device)
            sgd = dict(w=sp.master.data_ptr() + 4 * s0, mom=None if mom is None else mom.data_ptr() + 4 * s0,
                       lr=lr, first=first, wd=g["weight_decay"], momentum=g["momentum"], dampening=g["dampening"],
                       nesterov=int(g["nesterov"]), grad_scale=1.0 / self.world)
            ready, wait, done, word, adv = 2 * seg + 1, 2 * seg + 1, 2 * seg + 2, 5 + seg, 0
        elif kind == "ag":
            a, b = ch, s1 - s0
            nv = (self.world - 1) * (ch * 2 // 16)
            data = arr(*[int(v) + 2 * s0 for v in self._shadows])
            sgd = dict(w=None, mom=None, lr=None, first=None, wd=0.0, momentum=0.0, dampening=0.0, nesterov=0,
                       grad_scale=1.0)
            last = seg == self.RIDER_STAGES - 1
            ready, wait, done, word, adv = 0, 2 * seg + 2, 0, 7, (4 if last else 0)
            if not last:
                word = 0      # no completion count for the first stage's gather
        else:
            raise ValueError(f"rider kind {kind!r}")
        cuts = [nv * i // n_hosts for i in range(n_hosts + 1)]
        total = n_hosts * blocks if word else 0
        # READY: every slice publishes it (block 0) — the backward runs the hosts in an order these
        # slices do not know, and a slice may only wait for what an earlier launch published
        return [ShardRider(self, 1 if kind == "rs" else 2, data, a, b, cuts[i], cuts[i + 1], ready, wait, done,
                           total, word if word else 5, adv, sp.shadow.data_ptr() + 2 * s0, blocks, sgd)
                for i in range(n_hosts)]

    def gather_master(self, max_blocks: int = 256):
        """Collective: complete the fp32 master from the owners' chunks.  Entry barrier, gather,
        then an exit barrier: callers overwrite their own master chunk right after this (tail
        local rounds, the next epoch's broadcast, the self-test restore), which must not happen
        while a slower peer is still reading that chunk."""
        if len(self.segments) == 1:
            HIP.call("kml_zs_all_gather", "p p p p i i l l i i i i d i p s", ctypes.addressof(self._flags),
                     ctypes.addressof(self._states), self.region, self.ctrl, self.rank, self.world, self.n,
                     self.chunk, 4, 1, 2, int(max_blocks), self.timeout_s, int(self.split), None, self._stream())
        else:
            last = len(self.segments) - 1
            for k, (s0, s1, ch) in enumerate(self.segments):
                _, st = self._seg_ptrs[k]
                HIP.call("kml_zs_all_gather", "p p p p i i l l i i i i d i p s", ctypes.addressof(self._flags),
                         ctypes.addressof(st), self.region, self.ctrl, self.rank, self.world, s1 - s0, ch, 4, 1,
                         2 if k == last else 1, int(max_blocks), self.timeout_s, int(self.split), None, self._stream())
        HIP.call("kml_zs_barrier", "p p p i i i d s", ctypes.addressof(self._flags), self.region, self.ctrl,
                 self.rank, self.world, 0, self.timeout_s, self._stream())
        self.space._master_stale = False

    # ------------------------------------------------------------------ health
    def errors(self) -> int:
        if self.ctrl is None:
            return 0
        out = ctypes.c_uint(0)
        HIP.call("kml_peer_errors", "p p", self.ctrl, ctypes.addressof(out))
        return int(out.value)

    def check(self):
        n = self.errors()
        if n:
            raise PeerCommError(f"sharded update: {n} barrier wait(s) on rank {self.rank}/{self.world} timed out "
                                f"after {self.timeout_s:g} s (a peer stopped calling); results since then are NaN")

    def self_test(self) -> bool:
        """Collective: reduce-scatter / gather the space's own buffers on rank-dependent integer
        patterns (exact in fp32 and bf16), compare with the closed forms, restore the buffers.
        True on every rank only if every rank was exact and no wait timed out."""
        sp = self.space
        ok = True
        saved = [t.clone() for t in (sp.grad, sp.shadow, sp.state)]
        try:
            idx = torch.arange(self.n, device=self.device)
            base = (idx % 8).float()
            sp.grad.copy_(base * float(self.rank + 1))
            self.reduce_scatter()
            tri = float(self.world * (self.world + 1) // 2)
            ok = ok and bool(torch.equal(sp.grad[self.lo:self.hi], base[self.lo:self.hi] * tri))
            owner = torch.div(idx, self.chunk, rounding_mode="floor").float()
            sp.shadow.copy_(((owner == self.rank).float() * (base + owner)).to(torch.bfloat16))
            self.all_gather_shadow()
            ok = ok and bool(torch.equal(sp.shadow.float(), base + owner))
            sp.master.copy_((owner == self.rank).float() * (base * 3 + owner))
            self.gather_master()
            ok = ok and bool(torch.equal(sp.master, base * 3 + owner))
            torch.cuda.synchronize(self.device)
            ok = ok and self.errors() == 0
            from ..utils import fault
            fault.point("shard_selftest", rank=self.rank)    # failure-path tests: this rank's check fails
        except Exception:
            ok = False
        finally:
            for t, s in zip((sp.grad, sp.shadow, sp.state), saved):
                t.copy_(s)
            sp._master_stale = False
            torch.cuda.synchronize(self.device)
        flags: List[bool] = [False] * self.world
        self.dist.all_gather_object(flags, ok, group=self.group)
        return all(flags)

    def set_fresh(self, ranges):
        """Flat [lo, hi) ranges whose fp32 master every rank's step reads (BN / LN affine, biases:
        nn ``master_of``).  The ZeRO-1 layout keeps a rank's master current only on its own chunks,
        so :meth:`gather_fresh` re-reads these elements from their owners after each step."""
        idx = [torch.arange(int(lo), int(hi), dtype=torch.int32) for lo, hi in ranges if hi > lo]
        self._fresh = torch.cat(idx).to(self.device) if idx else None

    def gather_fresh(self):
        """Stream-ordered, capturable: the :meth:`set_fresh` elements owned elsewhere := their
        owners' fp32 master (csrc/kernels/comm.hip k_zs_fresh).  Call after the step's last
        all-gather."""
        fresh = getattr(self, "_fresh", None)
        if self.world == 1 or fresh is None or fresh.numel() == 0:
            return
        if self.region is None:
            raise PeerCommError("sharded update used after close()")
        segs = (ctypes.c_longlong * (3 * len(self.segments)))(*[int(v) for seg in self.segments for v in seg])
        HIP.call("kml_zs_fresh", "p l p i i p i s", fresh.data_ptr(), int(fresh.numel()),
                 ctypes.addressof(self._states), self.rank, self.world, ctypes.addressof(segs), len(self.segments),
                 self._stream())

    def rider_self_test(self, riders, optimizer) -> bool:
        """Collective: every rider slice (:meth:`rider_slices`, in phase order) run once on its own
        launch on rank-dependent integer gradients with the master zeroed, lr = -1 and the first
        momentum step, so each owner's master chunk becomes the rank-ordered gradient mean (times
        1 + momentum with Nesterov) and every shadow of the riding stages its bf16; compared with
        the closed form, then every touched buffer restored.  True on every rank only if every rank
        was exact and no wait timed out (engine/dp.py then keeps the riders, else the plain shard
        step)."""
        sp = self.space
        g = optimizer.param_groups[0]
        mom = optimizer._bufs(sp, ["momentum"])["momentum"] if g["momentum"] != 0 else None
        lr = optimizer.lr_tensor(sp.device)
        first = optimizer.first_tensor(sp.device) if mom is not None else None
        keep = [sp.grad, sp.shadow, sp.master, lr] + ([mom, first] if mom is not None else [])
        saved = [t.clone() for t in keep]
        ok = True
        try:
            idx = torch.arange(self.n, device=self.device)
            base = (idx % 8).float()
            sp.grad.copy_(base * float(self.rank + 1))
            sp.master.zero_()
            lr.fill_(-1.0)
            if mom is not None:
                mom.zero_()
                first.fill_(1.0)
            for r in riders:
                r.run_alone()
            torch.cuda.synchronize(self.device)
            d = (base * float(self.world * (self.world + 1) // 2)) * (1.0 / self.world)
            want = d + g["momentum"] * d if (mom is not None and g["nesterov"]) else d
            for k in range(min(self.RIDER_STAGES, len(self.segments))):
                s0, s1, ch = self.segments[k]
                lo = min(s1, s0 + self.rank * ch)
                hi = min(s1, lo + ch)
                ok = ok and bool(torch.allclose(sp.master[lo:hi], want[lo:hi], rtol=1e-6, atol=0))
                ok = ok and bool(torch.equal(sp.shadow[s0:s1].float(), want[s0:s1].to(torch.bfloat16).float()))
            ok = ok and self.errors() == 0
            from ..utils import fault
            fault.point("rider_selftest", rank=self.rank)    # failure-path tests: this rank's check fails
        except Exception:
            ok = False
        finally:
            for t, v in zip(keep, saved):
                t.copy_(v)
            torch.cuda.synchronize(self.device)
        flags: List[bool] = [False] * self.world
        self.dist.all_gather_object(flags, ok, group=self.group)
        return all(flags)

    def _release(self):
        for p in self.opened:
            try:
                HIP.call("kml_ipc_close", "p", p)
            except Exception:
                pass
        self.opened = []
        if self.region is not None:
            HIP.call("kml_peer_free", "p p", self.region, self.ctrl)
        self.region = self.ctrl = None
        if getattr(self.space, "master_sync", None) == self.gather_master:
            self.space.master_sync = None

    def close(self):
        """Collective over the group: unmap the peers' buffers once everyone is done."""
        if self.region is None:
            return
        torch.cuda.synchronize(self.device)
        self.dist.barrier(group=self.group)
        self._release()
        self.dist.barrier(group=self.group)


class ShardRider:
    """One peer-shard slice carried by a later backward launch (csrc/include/kml_sgd.h KmlZsRider:
    the conv pair's rider blocks, or its own launch when the host took another path): the same
    arm() / run_alone() protocol as :class:`~kubeml_amd.ops.kernels.SgdRider`."""

    def __init__(self, shard, kind, data, a, b, v0, v1, ready, wait, done, done_blocks, done_word, advance, shadow,
                 blocks, sgd):
        self.shard, self.kind, self.data = shard, kind, data
        self.a, self.b, self.v0, self.v1 = int(a), int(b), int(v0), int(v1)
        self.ready, self.wait, self.done = int(ready), int(wait), int(done)
        self.done_blocks, self.done_word, self.advance = int(done_blocks), int(done_word), int(advance)
        self.shadow, self.blocks, self.sgd = int(shadow), int(blocks), sgd

    def arm(self):
        sh, g = self.shard, self.sgd
        if sh.region is None:
            raise PeerCommError("shard rider used after close()")
        HIP.call("kml_zs_rider_set", "i p p p p i i l l l l i i i i i i d p p p p p f f f i f i", self.kind,
                 ctypes.addressof(sh._flags), ctypes.addressof(self.data), sh.region, sh.ctrl, sh.rank, sh.world,
                 self.a, self.b, self.v0, self.v1, self.ready, self.wait, self.done, self.done_blocks,
                 self.done_word, self.advance, sh.timeout_s, g["w"], g["mom"], self.shadow,
                 None if g["lr"] is None else g["lr"].data_ptr(),
                 None if g["first"] is None else g["first"].data_ptr(), float(g["wd"]), float(g["momentum"]),
                 float(g["dampening"]), int(g["nesterov"]), float(g["grad_scale"]), self.blocks)

    def run_alone(self):
        """The same slice as its own launch (its host took a path without a rider role)."""
        self.arm()
        HIP.call("kml_rider_flush", "s", torch.cuda.current_stream(self.shard.device).cuda_stream)


def verified_shard(space, group=None, log=None) -> Optional[PeerShard]:
    """Collective: a :class:`PeerShard` that passed its self-test on every rank, or None on every
    rank (callers then use the all-reduce plans).  ``KUBEML_PEER_SELFTEST=0`` skips the test."""
    try:
        p = PeerShard(space, group)
    except PeerCommError as e:
        if log:
            log(f"sharded update unavailable: {e}")
        return None
    if os.environ.get("KUBEML_PEER_SELFTEST", "1") == "0" or p.self_test():
        return p
    if log:
        log("sharded update failed its self-test on this node")
    try:
        p.close()
    except Exception:
        pass
    return None


def stream_copy(src: torch.Tensor, dst: torch.Tensor, nbytes: int, blocks: int, passes: int = 1):
    """Interference-probe streamer: ``passes`` copies of ``nbytes`` on ``blocks`` workgroups."""
    HIP.call("kml_stream_copy", "p p l i i s", src.data_ptr(), dst.data_ptr(), int(nbytes), int(blocks), int(passes),
             torch.cuda.current_stream(src.device).cuda_stream)


def stamp(buf: torch.Tensor, idx: int):
    """Device wall-clock stamp (100 MHz ticks) into ``buf[idx]`` (int64) on the current stream."""
    if not (buf.is_cuda and buf.dtype == torch.int64 and 0 <= idx < buf.numel()):
        raise ValueError("stamp: int64 CUDA buffer and an index inside it")
    HIP.call("kml_stamp", "p i s", buf.data_ptr(), int(idx), torch.cuda.current_stream(buf.device).cuda_stream)
