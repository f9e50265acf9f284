"""Graph-captured data-parallel training step (the hot loop of a resident GPU worker).

One training step of a CNN workload on an MI355X is ~200 small kernels (ResNet-34 at
32x32: GEMMs of a few GFLOP each).  Launched from Python that is host-bound, so the
step is captured ONCE into a hipGraph (``torch.cuda.graph``) and replayed:

    segment 0 .. S-1 :  [pre: augment batch, zero grads] forward, loss, backward split
                        into S segments; after segment k its finished gradient range is
                        all-reduced (SUM, RCCL over xGMI) while segment k+1 computes
    optimizer        :  fused SGD/Adam over the flat buffer (1/world folded in)

With one rank everything is one graph.  With several, the collectives are either
captured into the same graph (``graph_comm``: one replay per step, RCCL kernels on the
process group's stream forked from / joined into the capture stream) or issued eagerly
between per-segment graph replays.  Everything that changes per step (data offset,
crop RNG, LR, Adam step, SGD first-step flag) lives in device memory, so replays are
exact re-executions with fresh data.

Capture never changes training state: the warm-up iterations that initialise the
allocator pool run WITHOUT collectives and on snapshots — every tensor in
``state_tensors`` (master weights, bf16 shadow, BN statistics and counters, optimizer
buffers and device scalars, data counters) is restored afterwards, so the first
``__call__`` is the first real update (reference semantics: one optimizer step per
minibatch, python/kubeml/kubeml/network.py:291-295).

This replaces the reference's per-iteration HTTP fan-out + Redis weight round-trip
(ml/pkg/train/job.go:295-334, python/kubeml/kubeml/network.py:252-310) for the K=1
(synchronous DP) case; K-step model averaging lives in :mod:`kubeml_amd.parallel.kavg`.
"""
from __future__ import annotations

import contextlib
import gc
from typing import Callable, List, Optional, Sequence

import torch
import torch.distributed as dist

from ..utils import trace


@contextlib.contextmanager
def capture_graph(g, **kw):
    """torch.cuda.graph with the cyclic garbage collected first and the collector paused for the
    capture: a collection inside the capture can free an earlier step's graph, events or
    library handles, and those destroy calls invalidate a global-mode capture."""
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        with torch.cuda.graph(g, **kw):
            yield
    finally:
        if was:
            gc.enable()


def train_state_tensors(module=None, space=None, optimizer=None, extra: Sequence[torch.Tensor] = ()):
    """Device tensors a training step mutates (for snapshot/restore around warm-up)."""
    out: List[torch.Tensor] = []
    seen = set()

    def add(t):
        if t is None or not isinstance(t, torch.Tensor) or t.numel() == 0:
            return
        key = (t.data_ptr(), t.numel(), t.dtype)
        if key not in seen:
            seen.add(key)
            out.append(t)
    if space is not None:
        add(getattr(space, "state", None) if getattr(space, "state", None) is not None else space.master)
        add(space.shadow)
        if hasattr(space, "i64_arena_now"):
            add(space.i64_arena_now())
    if module is not None:
        state = getattr(space, "state", None) if space is not None else None
        lo = state.data_ptr() if state is not None else -1
        hi = lo + state.numel() * 4 if state is not None else -1
        for b in module.buffers():
            if b is not None and not (lo <= b.data_ptr() < hi):
                add(b)
        arena = getattr(module, "_nbt_arena", None)
        add(arena)
    if optimizer is not None and hasattr(optimizer, "state_tensors"):
        if hasattr(optimizer, "prepare"):
            optimizer.prepare()
        for t in optimizer.state_tensors():
            add(t)
    for t in extra:
        add(t)
    return out


def _narrow(v, lp):
    """fp32 gradient range -> bf16 communication buffer (HIP kernel on the GPU)."""
    if v.is_cuda:
        from ..ops import kernels as K
        K.f32_to_bf16(v, out=lp)
    else:
        lp.copy_(v.reshape(-1))


def _widen(lp, v):
    if v.is_cuda:
        from ..ops import kernels as K
        K.bf16_to_f32(lp, out=v)
    else:
        v.reshape(-1).copy_(lp)


class _SideJoin:
    """'Work' handle of a side-stream collective: waiting joins the side stream into the
    current one (a graph join edge when captured)."""

    def __init__(self, side):
        self.side = side

    def wait(self):
        torch.cuda.current_stream(self.side.device).wait_stream(self.side)


class _Snapshot:
    def __init__(self, tensors):
        self.tensors = list(tensors)
        self.copies = [t.detach().clone() for t in self.tensors]

    def restore(self):
        with torch.no_grad():
            for t, c in zip(self.tensors, self.copies):
                t.copy_(c)
        self.copies = []


class GraphedTrainStep:
    """Captures forward/backward segments (+ collectives) + optimizer into hipGraphs.

    fwd_bwd: callable running forward+backward and returning the loss tensor (device);
        used when ``segments`` is None (one segment whose gradients are ``grad_buffers``)
    opt_step: callable applying the optimizer (+ any counter advance)
    grad_buffers: flat fp32 gradient tensors all-reduced (SUM) after fwd_bwd
    segments / segment_grads: ``segments[0]`` is forward + the first part of backward
        (returns the loss), ``segments[k]`` continue backward; ``segment_grads[k]`` lists
        the gradient views that are final after segment ``k``.
    state_tensors: tensors restored after the warm-up (see module docstring)
    graph_comm: capture the collectives into the step's graph (one replay per step)
    bucket_mb: split each all-reduce into buckets of at most this size (0 = whole views)
    comm_dtype: torch.float32 (default) or torch.bfloat16 — gradient compression: each
        finished gradient range is rounded to a persistent bf16 buffer, all-reduced in bf16
        (half the xGMI bytes), and widened back into the fp32 gradient before the optimizer
        (the fused optimizer still applies the 1/P scale in fp32).  Opt-in: the SUM of P
        bf16 values carries bf16 rounding (~3 significant digits) into the update.
    """

    def __init__(self, fwd_bwd: Optional[Callable[[], torch.Tensor]], opt_step: Callable[[], None],
                 grad_buffers=(), group=None, use_graph: bool = True, warmup: int = 1, bucket_mb: float = 0.0,
                 segments=None, segment_grads=None, force_comm: bool = False, graph_comm: bool = True,
                 state_tensors: Sequence[torch.Tensor] = (), comm_dtype=torch.float32,
                 segment_opt: Optional[Sequence[Callable[[], None]]] = None,
                 opt_finish: Optional[Callable[[], None]] = None, peer=None, schedule: str = "overlap",
                 peer_blocks: int = 256, comm_timing: int = 0, shard_step: Optional[Callable[[], None]] = None,
                 on_replay: Optional[Callable[[], None]] = None, world: Optional[int] = None,
                 segment_shard: Optional[Sequence[Callable]] = None):
        if segments is None:
            if fwd_bwd is None:
                raise ValueError("need fwd_bwd or segments")
            segments = [fwd_bwd]
            segment_grads = [list(grad_buffers)]
        self.segments = list(segments)
        self.segment_grads = [list(g) for g in segment_grads] if segment_grads else [[] for _ in self.segments]
        if len(self.segment_grads) != len(self.segments):
            raise ValueError("segment_grads must have one entry per segment")
        self.opt_step = opt_step
        self.group = group
        # world: ranks of THIS step's gradient exchange.  Given explicitly by make_train_step: a
        # local step (world 1) of a process that belongs to a larger default group must not
        # reduce over that group
        if world is None:
            world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.world = int(world)
        # force_comm: issue the collectives even on a 1-rank group (exercises RCCL next to
        # the captured graphs on a single-GPU box)
        self.comm = self.world > 1 or (force_comm and dist.is_available() and dist.is_initialized())
        self._comm_on = True
        self.graph_comm = graph_comm
        self.use_graph = use_graph
        self.warmup = warmup
        self.bucket_elems = int(bucket_mb * 2**20 / 4) if bucket_mb > 0 else 0
        self.state_tensors = list(state_tensors)
        if comm_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("comm_dtype must be torch.float32 or torch.bfloat16")
        self.comm_dtype = comm_dtype
        self._lp = {}      # fp32 view key -> persistent bf16 communication buffer
        self._pending_widen = []
        # optimizer overlapped with backward: segment_opt[k] applies the update to segment
        # k's (final, all-reduced) gradients on a side stream; opt_finish closes the step
        if segment_opt is not None and (len(segment_opt) != len(self.segments) or opt_finish is None):
            raise ValueError("segment_opt needs one callable per segment and opt_finish")
        self.segment_opt = list(segment_opt) if segment_opt is not None else None
        self.opt_finish = opt_finish
        self._opt_side = None
        # peer backend (parallel/peer.py): plain kernels, so the collectives always live in
        # the step's one graph; "end" = one all-reduce per view after the whole backward on
        # the compute stream, "overlap" = per segment on a side stream (block-capped)
        if schedule not in ("end", "overlap", "shard"):
            raise ValueError("schedule must be 'end', 'overlap' or 'shard'")
        if schedule == "shard" and shard_step is None:
            raise ValueError("the shard schedule needs shard_step (reduce-scatter, update, all-gather)")
        self.peer = peer if self.comm else None
        self.schedule = schedule
        # shard: the optimizer is part of the collective (parallel/peer.py PeerShard) — with the
        # collectives on, shard_step replaces opt_step; the local warm-up still runs opt_step
        self.shard_step = shard_step if self.comm else None
        self.on_replay = on_replay      # host bookkeeping after every replay (e.g. master now sharded)
        # staged shard ("shardov"): segment_shard[k](stamps) = stage k's reduce-scatter + SGD +
        # all-gather, issued on a block-capped side stream right after segment k's backward
        if segment_shard is not None and (shard_step is None or len(segment_shard) != len(self.segments)):
            raise ValueError("segment_shard needs shard_step and one callable per segment")
        self.segment_shard = list(segment_shard) if (segment_shard is not None and self.comm) else None
        self._shard_side = None
        self.peer_blocks = int(peer_blocks)
        self._peer_side = None
        if self.peer is not None and self.segment_opt is not None:
            raise ValueError("the peer backend does not combine with the per-segment optimizer overlap")
        # comm_timing = T > 0: every T-th replay records HIP events around the collectives
        # (a separate graph with event nodes), read back lazily -> comm_seconds()
        self.comm_timing = int(comm_timing)
        self._replays = 0
        self._timed = None          # (graph, [(start, end) events]) of the timed variant
        self._pending_times = []
        self.comm_time_total = 0.0
        self.comm_time_samples = 0
        self._dev = next((t.device for g in self.segment_grads for t in g), None)
        self._stamps = self._host_stamps = self._pending_stamp = None
        if self.comm_timing and self.comm and self._dev is not None and self._dev.type == "cuda":
            # allocated here, never inside a capture
            self._stamps = torch.zeros(2, dtype=torch.int64, device=self._dev)
            self._host_stamps = torch.zeros(2, dtype=torch.int64).pin_memory()
        self.g_seg: List[torch.cuda.CUDAGraph] = []
        self.g_all = None
        self.g_opt = None
        self.loss = None
        self.captured = False

    # ------------------------------------------------------------------ pieces
    @staticmethod
    def _run(fn):
        """Run one forward/backward segment callable."""
        return fn()

    def _views(self, k):
        for t in self.segment_grads[k]:
            if not t.numel():
                continue
            if self.bucket_elems and t.numel() > self.bucket_elems:
                for s in range(0, t.numel(), self.bucket_elems):
                    yield t[s:s + self.bucket_elems]
            else:
                yield t

    def _lp_buf(self, v):
        key = (v.data_ptr(), v.numel())
        b = self._lp.get(key)
        if b is None or b.device != v.device:
            b = self._lp[key] = torch.empty(v.numel(), dtype=torch.bfloat16, device=v.device)
        return b

    # ------------------------------------------------------------------ comm timing
    def _stamp(self, idx, dev):
        """Device wall-clock stamp of the collectives' start (0) / end (1) on the current
        stream (only when ``comm_timing`` is on)."""
        if self._stamps is None:
            return
        from ..parallel.peer import stamp
        stamp(self._stamps, idx)

    def _sample_comm_time(self):
        """After a replay: every ``comm_timing``-th step copy the stamps to pinned memory
        (non-blocking) and fold the previous sample in once its copy has landed."""
        if self._stamps is None:
            return
        self._replays += 1
        self._fold_stamp()
        if self._pending_stamp is None and self._replays % self.comm_timing == 0:
            self._host_stamps.copy_(self._stamps, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._pending_stamp = ev

    def _fold_stamp(self):
        pend = self._pending_stamp
        if pend is not None and pend.query():
            t0, t1 = self._host_stamps.tolist()
            if t1 >= t0:
                self.comm_time_total += (t1 - t0) / 1e8      # s_memrealtime: 100 MHz
                self.comm_time_samples += 1
            self._pending_stamp = None

    def comm_seconds(self) -> float:
        """Mean seconds of one step's gradient collectives over the sampled steps (0.0 if
        unsampled).  Peer/end: the all-reduce itself (peer wait included); overlap: from the
        first segment's collective to the last one's completion."""
        if self._stamps is not None:
            self._fold_stamp()          # a sample whose copy has landed since the last replay
        return self.comm_time_total / self.comm_time_samples if self.comm_time_samples else 0.0

    # ------------------------------------------------------------------ collectives
    def _peer_call(self, v):
        self.peer.all_reduce_(v, algo="twoshot", wire=self.comm_dtype, max_blocks=self.peer_blocks)

    def _issue(self, k):
        """Async all-reduce of the gradients finished by segment k (bf16-compressed with
        ``comm_dtype=torch.bfloat16``: the widening back runs in :meth:`_finish_comm`)."""
        if not (self.comm and self._comm_on) or self.shard_step is not None:
            return []
        views = list(self._views(k))
        if not views:
            return []
        if self.peer is not None:
            if self.schedule == "end":
                return []                     # all views go after the backward (_finish_comm)
            cur = torch.cuda.current_stream(views[0].device)
            if self._peer_side is None:
                self._peer_side = torch.cuda.Stream(views[0].device)
            side = self._peer_side
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                if k == 0:
                    self._stamp(0, views[0].device)
                for v in views:
                    self._peer_call(v)
                if k == len(self.segments) - 1:
                    self._stamp(1, views[0].device)
            return [_SideJoin(side)]
        if k == 0:
            self._stamp(0, views[0].device)
        if self.comm_dtype == torch.float32:
            return [dist.all_reduce(v, group=self.group, async_op=True) for v in views]
        works = []
        for v in views:
            lp = self._lp_buf(v)
            _narrow(v, lp)
            works.append(dist.all_reduce(lp, group=self.group, async_op=True))
            self._pending_widen.append((lp, v))
        return works

    def _finish_comm(self, works):
        if self.peer is not None and self.schedule == "end" and self.comm and self._comm_on:
            views = [v for k in range(len(self.segments)) for v in self._views(k)]
            if views:
                self._stamp(0, views[0].device)
                for v in views:
                    self._peer_call(v)
                self._stamp(1, views[0].device)
        for w in works:
            w.wait()
        for lp, v in self._pending_widen:
            _widen(lp, v)
        self._pending_widen = []
        if self.peer is None and works and self.comm and self._comm_on and self._dev is not None:
            self._stamp(1, self._dev)

    def _body(self):
        if self.segment_opt is not None:
            return self._body_opt_overlap()
        if self.segment_shard is not None and self._comm_on:
            return self._body_staged_shard()
        loss, works = None, []
        for k, seg in enumerate(self.segments):
            out = self._run(seg)
            if k == 0:
                loss = out
            works += self._issue(k)
        self._finish_comm(works)
        if self.shard_step is not None and self._comm_on:
            self.shard_step(stamps=self._stamps)     # the collective's own launches stamp it
        else:
            self.opt_step()
        return loss

    def _body_staged_shard(self):
        """Staged ZeRO-1 step: after segment k's backward its gradient range is final, and
        stage k's reduce-scatter (peer reads over xGMI) + fused SGD + bf16 all-gather run on a
        side stream while segment k+1 (the stage before it) runs backward.  Stage k's weights
        are not read again this step, so updating them early is exact; the compute stream joins
        the side stream before the step ends (the next forward reads every stage)."""
        cur = torch.cuda.current_stream()
        if self._shard_side is None:
            self._shard_side = torch.cuda.Stream()
        side = self._shard_side
        loss = None
        for k, seg in enumerate(self.segments):
            out = self._run(seg)
            if k == 0:
                loss = out
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                if self._stamps is not None:
                    self.segment_shard[k]((self._stamps.data_ptr(), self._stamps.data_ptr() + 8))
                else:
                    self.segment_shard[k](None)
        cur.wait_stream(side)
        self.shard_step(stamps=None)
        return loss

    def _body_opt_overlap(self):
        """Per-segment update on a side stream: after segment k's backward (and its
        all-reduce, which the side stream waits for) the optimizer applies segment k's
        gradient range while segment k+1's backward runs; the compute stream joins the side
        stream before the step ends.  Segment k's weights are not read again this step
        (stage k's backward is complete), so updating them early is exact."""
        cur = torch.cuda.current_stream() if torch.cuda.is_available() else None
        side = None
        if cur is not None and any(t.is_cuda for g in self.segment_grads for t in g):
            if self._opt_side is None:
                self._opt_side = torch.cuda.Stream()
            side = self._opt_side
        loss = None
        for k, seg in enumerate(self.segments):
            out = self._run(seg)
            if k == 0:
                loss = out
            works = self._issue(k)
            if side is None:
                self._finish_comm(works)
                self.segment_opt[k]()
                continue
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                self._finish_comm(works)      # the side stream waits for this segment's all-reduce
                self.segment_opt[k]()
        if side is not None:
            cur.wait_stream(side)
        self.opt_finish()
        return loss

    def prime_comm(self):
        """One eager all-reduce of every gradient view (sets up RCCL connections before
        the first capture).  Call on ALL ranks at the same point."""
        if not self.comm or self.peer is not None or self.shard_step is not None:
            return
        for k in range(len(self.segments)):
            for v in self._views(k):
                dist.all_reduce(v if self.comm_dtype == torch.float32 else self._lp_buf(v), group=self.group)

    # ------------------------------------------------------------------ capture
    def capture(self):
        if not self.use_graph or not torch.cuda.is_available():
            return
        snap = _Snapshot(self.state_tensors) if self.state_tensors else None
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        self._comm_on = False            # warm-up: local only (peers are not stepping)
        try:
            with torch.cuda.stream(s):
                for _ in range(self.warmup):
                    self._body()
        finally:
            self._comm_on = True
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        if snap is not None:
            snap.restore()
            torch.cuda.synchronize()
        # with a process group alive, the RCCL watchdog thread polls work events while we
        # capture; "thread_local" keeps its (uncaptured) queries from invalidating the
        # capture.  Nothing on this thread makes an unsafe call inside a capture.
        mode = "thread_local" if self.comm else "global"
        if self.comm and trace.enabled() and self.shard_step is None:
            self.graph_comm = False   # keep the collectives outside the graph so they can be timed
        captured_all = False
        if not self.comm or self.graph_comm:
            try:
                g = torch.cuda.CUDAGraph()
                with capture_graph(g, capture_error_mode=mode):
                    self.loss = self._body()
                self.g_all, self.g_seg, self.g_opt = g, [], None
                captured_all = True
            except RuntimeError as e:
                if not self.comm or self.shard_step is not None:
                    raise
                import traceback
                traceback.print_exc()
                # the collectives would not capture on this RCCL/driver build: every rank hits
                # the same op, so all fall back together to per-segment graphs with eager
                # collectives between the replays
                import sys
                print(f"[kubeml] all-reduce capture failed ({str(e)[:200]}); falling back to per-segment "
                      f"graphs with eager collectives", file=sys.stderr, flush=True)
                torch.cuda.synchronize()
                self._pending_widen = []
                self.graph_comm = False
                self.graph_comm_fallback = True
                self.segment_opt = None       # per-segment graphs run the optimizer at the end
        if not captured_all:
            pool = torch.cuda.graph_pool_handle()
            self.g_seg = []
            for k, seg in enumerate(self.segments):
                g = torch.cuda.CUDAGraph()
                with capture_graph(g, pool=pool, capture_error_mode=mode):
                    out = self._run(seg)
                if k == 0:
                    self.loss = out
                self.g_seg.append(g)
            self.g_opt = torch.cuda.CUDAGraph()
            with capture_graph(self.g_opt, pool=pool, capture_error_mode=mode):
                self.opt_step()
            self.g_all = None
        torch.cuda.synchronize()
        self.captured = True

    def __call__(self):
        if self.on_replay is not None:
            self.on_replay()
        if not self.captured:
            self.loss = self._body()
            return self.loss
        if self.g_all is not None:
            if trace.enabled():
                e0 = trace.gpu_mark()
                self.g_all.replay()
                trace.gpu_span("step (one graph)", e0, trace.gpu_mark(), "gpu:compute")
            else:
                self.g_all.replay()
            self._sample_comm_time()
            return self.loss
        if trace.enabled():
            return self._traced_replay()
        works = []
        for k, g in enumerate(self.g_seg):
            g.replay()
            works += self._issue(k)
        self._finish_comm(works)
        self.g_opt.replay()
        return self.loss

    def _traced_replay(self):
        """Segment replays with device-timestamped spans: each segment on the compute
        track, each segment's all-reduce on the comm track from its issue point to its
        completion (observed by a side stream waiting on the collective), so a trace shows
        how much of the gradient traffic hides behind the next segment's backward."""
        cur = torch.cuda.current_stream()
        side = getattr(self, "_trace_side", None)
        if side is None:
            side = self._trace_side = torch.cuda.Stream()
        works = []
        for k, g in enumerate(self.g_seg):
            e0 = trace.gpu_mark(cur)
            g.replay()
            e1 = trace.gpu_mark(cur)
            trace.gpu_span(f"fwd+bwd seg{k}" if k == 0 else f"bwd seg{k}", e0, e1, "gpu:compute", segment=k)
            wk = self._issue(k)
            if wk:
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    for w in wk:
                        w.wait()
                    trace.gpu_span(f"allreduce seg{k}", e1, trace.gpu_mark(side), "gpu:comm", segment=k,
                                   bytes=sum(v.numel() * (4 if self.comm_dtype == torch.float32 else 2)
                                             for v in self._views(k)))
            works += wk
        self._finish_comm(works)
        e0 = trace.gpu_mark(cur)
        self.g_opt.replay()
        trace.gpu_span("optimizer", e0, trace.gpu_mark(cur), "gpu:compute")
        return self.loss
