"""Flat parameter space: one fp32 master / fp32 grad / bf16 shadow buffer per model.

Why flat (MI355X-first): the optimizer step, the gradient all-reduce over RCCL and
the K-AVG model average are then each ONE launch / ONE collective over a contiguous
buffer sized for HBM, instead of ~200 per-tensor launches.  This is the
equivalent of the reference's reference-model store (ml/pkg/model/model.go:14-53,
one gorgonia tensor per layer merged on the CPU), re-homed to HBM.

Layout rules
------------
* Every parameter owns a *storage region* whose shape is chosen by its module
  (conv weights: KRSC ``[Cout, KH, KW, Cin_pad]`` so the MFMA kernels read them
  directly) and is exposed to PyTorch as a strided *view* with the usual torch
  shape (``[Cout, Cin, KH, KW]``).  ``state_dict()`` therefore carries exactly the
  torchvision names and shapes, and torch optimizers / ``load_state_dict`` keep
  working.
* ``p.grad`` is bound to the matching view of the grad buffer with torch's
  zero-then-accumulate semantics, but the buffer is not memset every step: producers
  that can store (conv / linear weight gradients, BN dgamma/dbeta, the fused CE bias
  gradient) ask :func:`grad_out` whether to overwrite or add; ``zero_grad()`` zeroes only
  the regions whose producers can only add (learned from the previous backward), in one
  launch; ``finish_grads()`` zeroes any overwrite region nobody wrote this step.
* ``p._kml_shadow`` is the bf16 copy in storage layout that the forward kernels
  consume; it is refreshed by the fused optimizers, or lazily when ``p._version``
  moved (a foreign optimizer or ``load_state_dict`` wrote the master).
* Regions are packed in REVERSE registration order so that backward (which runs
  from the last layer to the first) fills the grad buffer front-to-back: a prefix
  of the buffer is final as soon as the corresponding layers are done, which is
  what the bucketed, backward-overlapped all-reduce exploits.
* Regions are 64-element aligned (256 B) so every region starts on a cache line.
* ``master`` is the head of a larger fp32 ``state`` buffer that also holds the
  module's floating-point buffers (BN running statistics, rebound as views), fp32
  slots for its int64 buffers (``num_batches_tracked``) and one participation-count
  slot: a K-AVG model average is then ONE all-reduce over ``state`` plus one fused
  scale kernel (parallel/kavg.py), instead of a per-round ``torch.cat`` of buffers.
"""
from __future__ import annotations

import os
from typing import Callable, Iterable, List, Optional

import torch

ALIGN = 64


def _storage_spec(p: torch.nn.Parameter):
    shape = getattr(p, "_kml_storage_shape", None)
    view = getattr(p, "_kml_view", None)
    if shape is None:
        return tuple(p.shape), (lambda s: s)
    return tuple(shape), view


class FlatParamSpace:
    """Owns the flat buffers for a list of parameters (all on one device)."""

    full_zero = False     # tests: memset the whole gradient every step (the reference behaviour)

    def __init__(self, params: Iterable[torch.nn.Parameter], device=None, reverse: bool = True,
                 with_shadow: Optional[bool] = None, buffers=None):
        """buffers: optional list of (module, name) of floating-point module buffers to
        place behind the parameters in ``state``; ``n_i64`` int64 buffers are given fp32
        slots via ``i64_buffers`` (list of (module, name))."""
        params = [p for p in params if p.requires_grad]
        seen = set()
        uniq = []
        for p in params:
            if id(p) not in seen:
                seen.add(id(p))
                uniq.append(p)
        self.params: List[torch.nn.Parameter] = list(reversed(uniq)) if reverse else uniq
        if device is None:
            device = self.params[0].device if self.params else torch.device("cpu")
        self.device = torch.device(device)
        if with_shadow is None:
            with_shadow = self.device.type == "cuda"
        self.offsets = []
        off = 0
        specs = []
        for p in self.params:
            shape, view = _storage_spec(p)
            n = 1
            for d in shape:
                n *= d
            specs.append((shape, view, n))
            self.offsets.append((off, n))
            off += -(-n // ALIGN) * ALIGN
        self.numel = max(off, ALIGN)
        fbufs, ibufs = buffers or ([], [])
        self.float_buffers = list(fbufs)
        self.i64_buffers = list(ibufs)
        boff = self.numel
        self.buffer_offsets = []
        for mod, name in self.float_buffers:
            n = getattr(mod, name).numel()
            self.buffer_offsets.append((boff, n))
            boff += n
        self.i64_off = -(-boff // 4) * 4
        self.n_i64 = len(self.i64_buffers)
        self.count_idx = self.i64_off + self.n_i64
        self.state_numel = -(-(self.count_idx + 1) // ALIGN) * ALIGN
        # GPU: state / grad / shadow each at the base of an IPC-exportable allocation, so the
        # peers of a data-parallel group can read them in place (parallel/peer.py PeerShard)
        bufs = None
        if self.device.type == "cuda" and with_shadow:
            from ..parallel.peer import ipc_zeros
            bufs = (ipc_zeros(self.state_numel, torch.float32, self.device),
                    ipc_zeros(self.numel, torch.float32, self.device),
                    ipc_zeros(self.numel, torch.bfloat16, self.device))
            if any(b is None for b in bufs):
                bufs = None
        self.ipc = bufs is not None
        if bufs is None:
            bufs = (torch.zeros(self.state_numel, dtype=torch.float32, device=self.device),
                    torch.zeros(self.numel, dtype=torch.float32, device=self.device),
                    torch.zeros(self.numel, dtype=torch.bfloat16, device=self.device) if with_shadow else None)
        self.state, self.grad, self.shadow = bufs
        self.master = self.state[:self.numel]
        # sharded (ZeRO-1) update: the fp32 master is complete only on this rank's chunk until
        # master_sync (the shard transport's gather) runs; see sync_master()
        self.master_sync = None
        self._master_stale = False
        with torch.no_grad():
            for p, (shape, view, n), (o, _) in zip(self.params, specs, self.offsets):
                st = self.master[o:o + n].view(shape)
                pv = view(st)
                pv.copy_(p.data.to(self.device))
                p.data = pv
                gst = self.grad[o:o + n].view(shape)
                p.grad = view(gst)
                p._kml_grad = p.grad
                p._kml_grad_storage = gst
                p._kml_master_storage = st
                if self.shadow is not None:
                    p._kml_shadow = self.shadow[o:o + n].view(shape)
                p._kml_flat = self
            for (mod, name), (o, n) in zip(self.float_buffers, self.buffer_offsets):
                b = getattr(mod, name)
                v = self.state[o:o + n].view(b.shape)
                v.copy_(b.to(self.device))
                setattr(mod, name, v)
        self.i64_arena = None
        if self.i64_buffers:
            self._bind_i64()
        self.refresh_shadow()
        self._index = {id(p): i for i, p in enumerate(self.params)}
        self._overwriters: set = set()   # param index -> its producer stored (grad_out) last backward
        self._accumulators: set = set()  # ... went through grad_storage_of (add-only producer)
        self._fresh: set = set()         # overwriters not yet written since zero_grad()
        self._zeroed_once = False
        self._folds: list = []           # (param, 1x1-form scratch, grad region, accumulate) to fold
        self._fold_cb = False            # an end-of-backward fold callback is queued

    def _bind_i64(self):
        """All int64 buffers as consecutive elements of one arena (one pointer for the
        K-AVG pack/finish kernels).  Models that keep their own arena (ResNet's packed
        ``num_batches_tracked``) are detected and reused."""
        ts = [getattr(m, n) for m, n in self.i64_buffers]
        base = ts[0]
        if all(t.numel() == 1 for t in ts) and all(
                t.data_ptr() == base.data_ptr() + 8 * i for i, t in enumerate(ts)):
            self.i64_arena = base.as_strided((len(ts),), (1,))
            return
        arena = torch.zeros(len(ts), dtype=torch.int64, device=self.device)
        with torch.no_grad():
            for i, ((m, n), t) in enumerate(zip(self.i64_buffers, ts)):
                arena[i] = t.reshape(()).to(self.device)
                setattr(m, n, arena[i])
        self.i64_arena = arena

    def i64_arena_now(self):
        """The int64 arena, re-detected if a model rebound its counters (e.g. on device move)."""
        if self.i64_buffers:
            ts = [getattr(m, n) for m, n in self.i64_buffers]
            a = self.i64_arena
            if a is None or any(t.data_ptr() != a.data_ptr() + 8 * i for i, t in enumerate(ts)):
                self._bind_i64()
        return self.i64_arena

    # ------------------------------------------------------------------ utilities
    def sync_master(self):
        """Complete a sharded fp32 master (collective over the shard group; no-op when every
        chunk is current).  Call before anything reads the full master: K-AVG, checkpoints,
        checksums."""
        if self._master_stale and self.master_sync is not None:
            self.master_sync()
        self._master_stale = False

    def refresh_shadow(self):
        """bf16 shadow := master (after init, load_state_dict, K-AVG averaging)."""
        if self.shadow is None:
            return
        if self.device.type == "cuda":
            from ..ops import kernels as K
            K.f32_to_bf16(self.master, self.shadow)
        else:
            self.shadow.copy_(self.master)
        for p in self.params:
            p._kml_shadow_version = p._version

    def rebind_grads(self):
        for p in self.params:
            p.grad = p._kml_grad

    def _region(self, i):
        o, n = self.offsets[i]
        return o, -(-n // ALIGN) * ALIGN

    def _zero_params(self, idx):
        """Zero the grad regions of the given parameter indices (merged runs, one launch per
        ``kml_zero_ranges_max()`` runs; the whole buffer when that is fewer launches)."""
        if not idx:
            return
        runs = []
        for i in sorted(idx):
            o, n = self._region(i)
            if runs and runs[-1][0] + runs[-1][1] == o:
                runs[-1][1] += n
            else:
                runs.append([o, n])
        from ..ops import kernels as K
        if len(runs) > K.zero_ranges_max():
            K.memset_(self.grad)
        else:
            K.zero_ranges_(self.grad, runs)

    def zero_grad(self):
        """torch semantics (every gradient reads as zero until its first producer writes),
        at the cost of zeroing only what an add-only producer will accumulate into."""
        if self.device.type != "cuda":
            self.grad.zero_()
        elif not self._zeroed_once or self.full_zero:
            from ..ops import kernels as K
            K.memset_(self.grad)          # first step: learn which producers overwrite
            self._zeroed_once = True
            self._fresh = set()
        else:
            self._zero_params([i for i in range(len(self.params)) if i not in self._overwriters])
            self._fresh = set(self._overwriters)
        self.rebind_grads()

    def grad_out(self, p) -> bool:
        """For a producer that can store: True = add to the region, False = overwrite it
        (the first write after zero_grad())."""
        i = self._index.get(id(p))
        if i is None:
            return True
        if i not in self._accumulators:
            self._overwriters.add(i)
        if i in self._fresh:
            self._fresh.discard(i)
            return False
        return True

    def grad_for_add(self, p):
        """For an add-only producer: make sure the region holds zeros if it is fresh, and
        remember that this parameter must be zeroed by zero_grad() from now on."""
        i = self._index.get(id(p))
        if i is None:
            return
        self._accumulators.add(i)
        self._overwriters.discard(i)
        if i in self._fresh:
            self._fresh.discard(i)
            self._zero_params([i])

    def defer_fold22(self, p, g):
        """An unrolled conv left its weight gradient in the dense 1x1 form in ``g``; fold it
        onto p's 3x3 taps at :meth:`finish_grads` (one launch for all of a stage's convs)."""
        dw, acc = grad_out(p)
        self._folds.append((p, g, dw, acc))
        if not self._fold_cb:
            # the folds also run when this backward pass ends, so .grad is final for any
            # reader (eager loops, tests); a later explicit finish_grads finds nothing left
            self._fold_cb = True
            torch.autograd.Variable._execution_engine.queue_callback(self._end_of_backward)

    def _end_of_backward(self):
        self._fold_cb = False
        if self._folds:
            self._run_folds(self._folds)
            self._folds = []

    def _run_folds(self, run):
        from ..ops import kernels as K
        K.fold22_multi([(g, dw, acc) for _, g, dw, acc in run])

    def finish_grads(self, params=None):
        """Make the gradients of ``params`` (all if None) final before they are consumed:
        run the deferred folds, zero the regions of overwrite parameters nobody wrote since
        zero_grad() (a parameter without a gradient this step)."""
        if self._folds:
            ids = None if params is None else {id(p) for p in params}
            run = [f for f in self._folds if ids is None or id(f[0]) in ids]
            if run:
                self._folds = [f for f in self._folds if not (ids is None or id(f[0]) in ids)]
                self._run_folds(run)
        if not self._fresh:
            return
        if params is None:
            left = set(self._fresh)
        else:
            left = {self._index[id(p)] for p in params if id(p) in self._index} & self._fresh
        self._fresh -= left
        self._zero_params(left)

    def finish_grads_range(self, start: int, end: int):
        """finish_grads for the parameters whose regions lie in flat elements [start, end)."""
        if self._fresh or self._folds:
            self.finish_grads([p for i, p in enumerate(self.params)
                               if start <= self.offsets[i][0] < end])

    def buckets(self, bucket_bytes: int):
        """Contiguous [start, end) element ranges of the grad buffer, ~bucket_bytes each,
        cut on parameter boundaries, in backward-completion order."""
        out = []
        cap = max(ALIGN, bucket_bytes // 4)
        start = 0
        cur_end = 0
        members = []
        for idx, (o, n) in enumerate(self.offsets):
            end = o + (-(-n // ALIGN) * ALIGN)
            members.append(idx)
            cur_end = end
            if cur_end - start >= cap:
                out.append((start, cur_end, members))
                start, members = cur_end, []
        if members:
            out.append((start, self.numel, members))
        return out

    def range_of(self, params) -> tuple:
        """[start, end) of the flat buffers covering exactly ``params`` (which must be
        contiguous in the layout: e.g. all parameters of a trailing group of layers)."""
        ids = {id(p) for p in params}
        idx = [i for i, p in enumerate(self.params) if id(p) in ids]
        if not idx:
            return (0, 0)
        if idx != list(range(idx[0], idx[-1] + 1)):
            raise ValueError("parameters are not contiguous in the flat layout")
        start = self.offsets[idx[0]][0]
        nxt = idx[-1] + 1
        end = self.offsets[nxt][0] if nxt < len(self.offsets) else self.numel
        return (start, end)

    def grad_view(self, params) -> torch.Tensor:
        s, e = self.range_of(params)
        return self.grad[s:e]

    def state_vector(self) -> torch.Tensor:
        return self.master


def module_buffers(module: torch.nn.Module, with_other: bool = False):
    """([(module, name)] of fp32 buffers, [(module, name)] of scalar int64 buffers) in
    ``named_buffers`` order; with ``with_other`` also the remaining persistent buffers (other
    floating dtypes, int32 / bool, non-scalar int64), which stay out of the fp32 state buffer
    and are averaged / broadcast through a side pack (parallel/kavg.py)."""
    fl, il, other = [], [], []
    for mod in module.modules():
        for name, b in mod._buffers.items():
            if b is None or name in getattr(mod, "_non_persistent_buffers_set", ()):
                continue
            if b.dtype == torch.float32:
                fl.append((mod, name))
            elif b.dtype == torch.int64 and b.numel() == 1:
                il.append((mod, name))
            else:
                other.append((mod, name))
    return (fl, il, other) if with_other else (fl, il)


def flatten_module(module: torch.nn.Module, device=None, buffers: bool = True) -> FlatParamSpace:
    """Move all trainable parameters (and, by default, the buffers) of ``module`` into
    one FlatParamSpace."""
    fl, il, other = module_buffers(module, with_other=True) if buffers else ([], [], [])
    space = FlatParamSpace(list(module.parameters()), device=device, buffers=(fl, il) if buffers else None)
    space.other_buffers = other      # not in ``state``: averaged / broadcast by a side pack
    module._kml_flat = space
    return space


def ensure_param_ready(p: torch.nn.Parameter):
    """Standalone (non-flattened) GPU parameter: give it grad/shadow storage once."""
    if getattr(p, "_kml_flat", None) is not None:
        return
    FlatParamSpace([p], device=p.device)


def shadow_of(p: torch.nn.Parameter) -> torch.Tensor:
    """bf16 storage-layout copy of p, refreshed if the master changed under us."""
    ensure_param_ready(p)
    if getattr(p, "_kml_shadow_version", None) != p._version:
        from ..ops import kernels as K
        st = p._kml_master_storage
        K.f32_to_bf16(st.contiguous(), p._kml_shadow)
        p._kml_shadow_version = p._version
    return p._kml_shadow


def grad_storage_of(p: torch.nn.Parameter) -> torch.Tensor:
    """fp32 storage-layout grad region of p for a producer that ADDS into it (zeroed if
    fresh, re-bound if p.grad was reset)."""
    ensure_param_ready(p)
    if p.grad is None:
        p._kml_grad_storage.zero_()
        p.grad = p._kml_grad
    p._kml_flat.grad_for_add(p)
    return p._kml_grad_storage


def grad_out(p: torch.nn.Parameter):
    """(fp32 storage-layout grad region, accumulate) for a producer that can either store
    (accumulate False: first write since zero_grad) or add."""
    ensure_param_ready(p)
    if p.grad is None:
        p._kml_grad_storage.zero_()
        p.grad = p._kml_grad
    return p._kml_grad_storage, p._kml_flat.grad_out(p)


def master_of(p: torch.nn.Parameter) -> torch.Tensor:
    """fp32 storage-layout master region of p (contiguous; what the kernels read)."""
    ensure_param_ready(p)
    return p._kml_master_storage


def grad_out_pair(p1: torch.nn.Parameter, p2: torch.nn.Parameter):
    """grad_out for two parameters one kernel writes with ONE store/add flag (BN dgamma and
    dbeta): (g1, g2, accumulate), the fresh one zeroed first if their states differ."""
    g1, a1 = grad_out(p1)
    g2, a2 = grad_out(p2)
    if a1 == a2:
        return g1, g2, a1
    fresh = p1 if not a1 else p2
    fresh._kml_flat._zero_params([fresh._kml_flat._index[id(fresh)]])
    return g1, g2, True
