"""Graph-captured data-parallel training step (the hot loop of a resident GPU worker).

One training step of a CNN workload on an MI355X is ~300 small kernels (ResNet-34 at
32x32: GEMMs of a few GFLOP each).  Launched from Python that is host-bound, so the
step is captured ONCE into a hipGraph (``torch.cuda.graph``) and replayed:

    segment A (graph):  augment batch -> zero grads -> forward -> loss -> backward
    all-reduce       :  flat fp32 gradient buffer, SUM over RCCL (xGMI), bucketed
    segment B (graph):  fused optimizer (1/world folded in) -> advance data counters

With world_size == 1 both segments are one graph.  Everything the step needs that
changes per step (data offset, crop RNG step, LR, Adam step) lives in device memory,
so replays are exact re-executions with fresh data, not stale copies.

This replaces the reference's per-iteration HTTP fan-out + Redis weight round-trip
(ml/pkg/train/job.go:295-334, python/kubeml/kubeml/network.py:252-310) for the K=1
(synchronous DP) case; K-step model averaging lives in :mod:`kubeml_amd.parallel.kavg`.
"""
from __future__ import annotations

import time
from typing import Callable, Optional

import torch
import torch.distributed as dist


class GraphedTrainStep:
    """Captures ``fwd_bwd()`` (+ ``opt_step()``) into hipGraphs around a DP all-reduce.

    fwd_bwd: callable running forward+backward and returning the loss tensor (device)
    opt_step: callable applying the optimizer (+ any counter advance)
    grad_buffers: list of flat fp32 gradient tensors to all-reduce (SUM) between them

    Overlapped mode (``segments`` + ``segment_grads``): ``segments[0]`` is forward +
    the first part of backward (returns the loss), ``segments[k]`` continue backward;
    ``segment_grads[k]`` lists the gradient views that are final after segment ``k``.
    Each segment is its own graph (shared pool); after replaying segment ``k`` the
    all-reduce of its gradients is issued asynchronously (RCCL on the process group's
    stream, ordered after the replay by an event) and the next segment's replay runs
    concurrently.  By default collectives are not captured: the multi-GPU path uses
    plain, eagerly-issued RCCL calls.  ``graph_comm=True`` instead captures the whole
    step, segments' all-reduces included (RCCL kernels on the process group's stream,
    forked from and joined back into the capture stream), into ONE graph: one replay
    per step, no host gaps between the segments.
    """

    def __init__(self, fwd_bwd: Callable[[], torch.Tensor], opt_step: Callable[[], None], grad_buffers=(),
                 group=None, use_graph: bool = True, warmup: int = 3, bucket_mb: float = 0.0,
                 segments=None, segment_grads=None, force_segments: bool = False, force_comm: bool = False,
                 graph_comm: bool = False):
        self.fwd_bwd = fwd_bwd
        self.opt_step = opt_step
        self.grad_buffers = list(grad_buffers)
        self.segments = list(segments) if segments else None
        self.segment_grads = [list(g) for g in segment_grads] if segment_grads else None
        self.force_segments = force_segments
        self.graph_comm = graph_comm
        self.g_seg = []
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        # force_comm: issue the collectives even on a 1-rank group (exercises RCCL next to
        # the captured graphs on a single-GPU box; the 8-GPU node is not ours to test on)
        self.comm = self.world > 1 or (force_comm and dist.is_available() and dist.is_initialized())
        self.use_graph = use_graph
        self.warmup = warmup
        self.bucket_elems = int(bucket_mb * 2**20 / 4) if bucket_mb > 0 else 0
        self.g_a = self.g_b = None
        self.loss = None
        self.captured = False

    @staticmethod
    def _run(fn):
        """Run a forward/backward callable with conv wgrads on the side stream (joined
        before returning, so a captured segment ends with all branches merged)."""
        from ..nn.fused import wgrad_overlap
        with wgrad_overlap():
            return fn()

    def _allreduce(self):
        if not self.comm:
            return
        for buf in self.grad_buffers:
            if self.bucket_elems and buf.numel() > self.bucket_elems:
                works = []
                for s in range(0, buf.numel(), self.bucket_elems):
                    works.append(dist.all_reduce(buf[s:s + self.bucket_elems], group=self.group, async_op=True))
                for w in works:
                    w.wait()
            else:
                dist.all_reduce(buf, group=self.group)

    def _eager(self):
        if self._segmented():
            loss = None
            works = []
            for k, seg in enumerate(self.segments):
                out = self._run(seg)
                if k == 0:
                    loss = out
                works += self._issue(k)
            for w in works:
                w.wait()
            self.opt_step()
            return loss
        loss = self._run(self.fwd_bwd)
        self._allreduce()
        self.opt_step()
        return loss

    def _segmented(self) -> bool:
        return self.segments is not None and (self.comm or self.force_segments)

    def _issue(self, k):
        """Async all-reduce of the gradients finished by segment k."""
        if not self.comm or not self.segment_grads:
            return []
        return [dist.all_reduce(t, group=self.group, async_op=True) for t in self.segment_grads[k] if t.numel()]

    def capture(self):
        if not self.use_graph or not torch.cuda.is_available():
            return
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(self.warmup):
                self._eager()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        # with a process group alive, the RCCL watchdog thread polls work events while we
        # capture; "thread_local" keeps its (uncaptured) queries from invalidating the
        # capture.  Nothing on this thread makes an unsafe call inside a capture.
        mode = "thread_local" if self.comm else "global"
        if self._segmented() and self.graph_comm and self.comm:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode=mode):
                works = []
                for k, seg in enumerate(self.segments):
                    out = self._run(seg)
                    if k == 0:
                        self.loss = out
                    works += self._issue(k)
                for w in works:
                    w.wait()
                self.opt_step()
            self.g_a, self.g_b, self.g_seg = g, None, []
        elif self._segmented():
            pool = torch.cuda.graph_pool_handle()
            self.g_seg = []
            for k, seg in enumerate(self.segments):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool, capture_error_mode=mode):
                    out = self._run(seg)
                if k == 0:
                    self.loss = out
                self.g_seg.append(g)
            self.g_b = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g_b, pool=pool, capture_error_mode=mode):
                self.opt_step()
        elif not self.comm:
            self.g_a = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g_a):
                self.loss = self._run(self.fwd_bwd)
                self.opt_step()
        else:
            self.g_a = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g_a, capture_error_mode=mode):
                self.loss = self._run(self.fwd_bwd)
            self.g_b = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g_b, capture_error_mode=mode):
                self.opt_step()
        torch.cuda.synchronize()
        self.captured = True

    def __call__(self):
        if not self.captured:
            self.loss = self._eager()
            return self.loss
        if self.g_seg:
            works = []
            for k, g in enumerate(self.g_seg):
                g.replay()
                works += self._issue(k)
            for w in works:
                w.wait()
            self.g_b.replay()
            return self.loss
        self.g_a.replay()
        if self.g_b is not None:
            self._allreduce()
            self.g_b.replay()
        return self.loss
