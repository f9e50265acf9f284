"""Stage-split forward/backward so gradient all-reduce overlaps the rest of backward.

A network is given as an ordered list of stages ``f_0 … f_{n-1}``.  The forward runs
all stages, cutting the autograd graph at each boundary (``h.detach().requires_grad_()``);
backward then runs stage by stage from the last:

    segment 0      : forward(all) -> loss -> backward(f_{n-1})       (grads of the tail)
    segment k (>0) : backward(f_{n-1-k}) from the boundary gradient

Each segment is a separately captured hipGraph (shared memory pool), so between
segment replays the DP step can launch the RCCL all-reduce of the gradients that
are already final (a contiguous range of the flat grad buffer, because the flat
layout stores parameters in reverse registration order) on the process-group stream,
while the next segment's backward keeps the CUs busy.  For ResNet-34 at batch 256 the
tail (fc + layer4 + layer3) holds 94 % of the 87 MB of gradients and the head
(stem, layer1, layer2) most of the backward FLOPs; with the head itself split at
layer1/layer2 only the stem + layer1 gradients (~1 MB) are all-reduced after the last
backward kernel, so almost the whole all-reduce hides behind compute — the MI355X/xGMI counterpart of DDP's bucketed overlap
(SURVEY §5.8 item 4).
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import torch


class StagedForwardBackward:
    def __init__(self, stages: Sequence[Callable], loss_fn: Callable, get_input: Callable,
                 pre: Optional[Callable] = None):
        """stages: callables h -> h; loss_fn(out) -> scalar loss; get_input() -> x;
        pre(): run at the start of segment 0 (zero grads, data augmentation, ...)."""
        self.stages = list(stages)
        self.loss_fn = loss_fn
        self.get_input = get_input
        self.pre = pre
        self._ins: List[Optional[torch.Tensor]] = []
        self._outs: List[Optional[torch.Tensor]] = []

    @property
    def n_segments(self) -> int:
        return len(self.stages)

    def segment(self, k: int):
        """Callable running segment ``k`` (0 returns the loss)."""
        if k == 0:
            return self._seg0
        return lambda: self._segk(k)

    def _seg0(self):
        if self.pre is not None:
            self.pre()
        h = self.get_input()
        n = len(self.stages)
        self._ins = [None] * n
        self._outs = [None] * n
        for i, st in enumerate(self.stages):
            if i > 0:
                h = h.detach().requires_grad_(True)
                self._ins[i] = h
            h = st(h)
            self._outs[i] = h
        loss = self.loss_fn(h)
        from ..nn.modules import backward_loss
        backward_loss(loss)
        return loss

    def _segk(self, k: int):
        i = len(self.stages) - 1 - k          # stage whose backward runs now
        g = self._ins[i + 1].grad
        self._outs[i].backward(g)
        if k == len(self.stages) - 1:
            self._ins = [None] * len(self.stages)   # drop references after the last segment
            self._outs = [None] * len(self.stages)

    def run_eager(self):
        loss = self._seg0()
        for k in range(1, self.n_segments):
            self._segk(k)
        return loss
