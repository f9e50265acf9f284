"""Synchronous data-parallel train step builder (north-star config 2).

One function, :func:`make_train_step`, assembles the framework's hot loop for a
flattened model: the (optionally stage-split) forward/backward, the backward-overlapped
gradient all-reduce over the job's RCCL group, the fused optimizer with the 1/P average
folded in, and the hipGraph capture that never mutates training state.  It is what
``KubeModel.step`` runs on resident GPU workers (sdk/model.py) and what the headline
``bench.py`` runs — the benchmark measures the framework's own path.

Reference: the per-iteration HTTP fan-out + Redis weight round trip of K=1 training
(ml/pkg/train/job.go:295-334, python/kubeml/kubeml/network.py:252-310).
"""
from __future__ import annotations

import os
from typing import Callable, Optional, Sequence

import torch

from .step import GraphedTrainStep, train_state_tensors


def make_train_step(model: torch.nn.Module, space, optimizer, loss_fn: Callable, x: torch.Tensor,
                    y: torch.Tensor, *, pre: Optional[Callable[[], None]] = None,
                    post: Optional[Callable[[], None]] = None, group=None, world: int = 1,
                    use_graph: bool = True, graph_comm: bool = True, overlap: bool = True,
                    bucket_mb: float = 0.0, force_comm: bool = False, warmup: int = 1,
                    extra_state: Sequence[torch.Tensor] = (), comm_dtype=None) -> GraphedTrainStep:
    """Build (not capture) the train step on static input buffers ``x``/``y``.

    pre():  runs first inside the step (e.g. on-device augmentation into ``x``)
    post(): runs after the optimizer (e.g. advance the data counter)
    world:  ranks in ``group``; > 1 adds the gradient all-reduce (SUM) and sets the
            optimizer's gradient scale to 1/world
    overlap: split backward at ``model.stages()`` (if the model has them) so each
            stage's gradients are all-reduced while the next stage's backward runs
    comm_dtype: torch.bfloat16 all-reduces bf16-rounded gradients (half the bytes; see
            :class:`GraphedTrainStep`); None = ``KUBEML_COMM_DTYPE`` (``bf16`` or fp32, default)
    """
    if comm_dtype is None:
        comm_dtype = torch.bfloat16 if os.environ.get("KUBEML_COMM_DTYPE", "fp32").lower() in (
            "bf16", "bfloat16") else torch.float32
    from ..nn import backward_loss
    comm = world > 1 or force_comm
    scale = 1.0 / max(world, 1)

    def opt_step():
        optimizer.set_grad_scale(scale)
        optimizer.step()
        if post is not None:
            post()

    segs = seg_grads = None
    if comm and overlap and hasattr(model, "stages") and hasattr(model, "stage_params"):
        from .staged import StagedForwardBackward

        def pre0():
            if pre is not None:
                pre()
            space.zero_grad()
        staged = StagedForwardBackward(model.stages(), lambda out: loss_fn(out, y), lambda: x, pre=pre0)
        segs = [staged.segment(k) for k in range(staged.n_segments)]
        sp = model.stage_params()
        seg_grads = [[space.grad_view(sp[len(sp) - 1 - k])] for k in range(len(sp))]
        fwd_bwd = None
    else:
        def fwd_bwd():
            if pre is not None:
                pre()
            space.zero_grad()
            loss = loss_fn(model(x), y)
            backward_loss(loss)
            return loss
    optimizer.set_grad_scale(scale)
    return GraphedTrainStep(fwd_bwd, opt_step, [space.grad], group=group, use_graph=use_graph, warmup=warmup,
                            bucket_mb=bucket_mb, segments=segs, segment_grads=seg_grads, force_comm=force_comm,
                            graph_comm=graph_comm, comm_dtype=comm_dtype,
                            state_tensors=train_state_tensors(model, space, optimizer, extra_state))
