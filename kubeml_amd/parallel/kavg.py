"""K-step model averaging (K-AVG / local SGD) — the reference's training algorithm.

Reference semantics:
* every worker trains on its shard for K local minibatch steps (K = -1: a whole epoch),
* then ALL model state (parameters and BN buffers, everything in ``state_dict``) is
  averaged over the workers that are still contributing (ml/pkg/model/model.go:249-302,
  parallelSGD.go:26-54; int64 buffers use integer division),
* each worker continues from the average and resets its optimizer state
  (python/kubeml/kubeml/network.py:121-128, 208-217).

MI355X-native: the average is ONE all-reduce over the flat fp32 parameter buffer
(RCCL over xGMI) plus one over a packed buffer of the BN running statistics, followed
by an in-place divide; the divisor is computed on the fly by a 1-element all-reduce,
so workers that ran out of data (uneven ``split_minibatches``) contribute zeros and are
excluded from the divisor, exactly like the reference's partial merge rounds.
"""
from __future__ import annotations

from typing import List, Tuple

import torch

from .comm import Comm


class ModelAverager:
    def __init__(self, module: torch.nn.Module):
        self.module = module

    def _param_tensors(self) -> List[torch.Tensor]:
        sp = getattr(self.module, "_kml_flat", None)
        if sp is not None:
            return [sp.master]
        out = []
        for p in self.module.parameters():
            if p.data.is_contiguous():
                out.append(p.data)
            else:
                out.append(p.data)  # handled by pack path below
        return out

    def _buffers(self) -> List[Tuple[str, torch.Tensor]]:
        return [(n, b) for n, b in self.module.named_buffers() if b is not None]

    @torch.no_grad()
    def average_(self, comm: Comm, participate: bool = True) -> int:
        if comm.world == 1:
            return 1 if participate else 0
        sp = getattr(self.module, "_kml_flat", None)
        bufs = self._buffers()
        params = [] if sp is not None else [p for p in self.module.parameters()]
        # pack everything that is not already one flat buffer into one fp32 vector
        pieces = [p.data.reshape(-1).float() for p in params] + [b.reshape(-1).double() if not b.is_floating_point()
                                                                  else b.reshape(-1).float() for _, b in bufs]
        dev = sp.master.device if sp is not None else (pieces[0].device if pieces else torch.device("cpu"))
        pack = torch.cat([x.float().to(dev) for x in pieces]) if pieces else None
        tensors = ([sp.master] if sp is not None else []) + ([pack] if pack is not None else [])
        n = comm.average_(tensors, participate)
        if n == 0:
            return 0
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
                b.copy_(torch.floor(v + 1e-6).to(b.dtype))
            off += k
        if sp is not None:
            sp.refresh_shadow()
        return n

    @torch.no_grad()
    def broadcast_(self, comm: Comm, src: int = 0):
        """Make every worker hold rank ``src``'s model (init / elastic scale-up)."""
        if comm.world == 1:
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
