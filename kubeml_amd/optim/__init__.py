"""Fused optimizers over the flat parameter space (one HIP launch per step).

``SGD`` / ``Adam`` / ``AdamW`` accept the same arguments as their ``torch.optim``
counterparts.  When the parameters live in :class:`~kubeml_amd.nn.flat.FlatParamSpace`
buffers (the GPU path) the step is one ``kml_sgd`` / ``kml_adam`` launch per space
that also refreshes the bf16 shadow copy; otherwise (CPU) it defers to the stock
torch implementation so CPU-only plumbing tests share the exact same semantics.

The learning rate lives in a device scalar (``lr_tensor``) so a graph-captured step
follows LR changes (``set_lr``) without re-capture, and Adam's step counter is a
device scalar incremented inside the captured region.

``reset_state()`` implements the reference's per-round optimizer reset under K-step
averaging (python/kubeml/kubeml/network.py:121-128): a memset of the state buffers,
Adam's device step counter back to 0 and SGD's device first-step flag back to 1 — all
read by the kernels at replay time, so a captured step honours a reset between replays.

``state_tensors()`` lists every device tensor a step mutates (state buffers, step
counters, flags); graph capture snapshots and restores them around its warm-up so
capturing a step never applies an update (engine/step.py).

``from_torch(opt)`` converts a user's ``torch.optim.SGD/Adam/AdamW`` (what
``KubeModel.configure_optimizers`` returns in reference code) into the fused one
with identical hyper-parameters.
"""
from __future__ import annotations

from typing import Dict, List

import torch

__all__ = ["SGD", "Adam", "AdamW", "from_torch", "FusedOptimizer"]


def _spaces(params):
    """Group params by their flat space (None for params without one)."""
    groups: Dict[int, tuple] = {}
    loose = []
    for p in params:
        sp = getattr(p, "_kml_flat", None)
        if sp is None:
            loose.append(p)
        else:
            groups.setdefault(id(sp), (sp, []))[1].append(p)
    return [g for g in groups.values()], loose


class FusedOptimizer(torch.optim.Optimizer):
    kind = "base"

    def __init__(self, params, defaults):
        super().__init__(params, defaults)
        self._state_bufs: Dict[int, Dict[str, torch.Tensor]] = {}
        self._lr_dev: Dict[torch.device, torch.Tensor] = {}
        self._grad_scale = 1.0
        self._first = True
        self._step_dev: Dict[torch.device, torch.Tensor] = {}
        self._first_dev: Dict[torch.device, torch.Tensor] = {}
        self._step_host = 0

    # --- device scalars -------------------------------------------------------------
    def lr_tensor(self, device):
        t = self._lr_dev.get(device)
        if t is None:
            t = torch.full((1,), float(self.param_groups[0]["lr"]), dtype=torch.float32, device=device)
            self._lr_dev[device] = t
        return t

    def set_lr(self, lr: float):
        for g in self.param_groups:
            g["lr"] = lr
        for t in self._lr_dev.values():
            t.fill_(float(lr))

    def set_grad_scale(self, s: float):
        """Folded into the step: the DP all-reduce SUMs, the optimizer averages."""
        self._grad_scale = float(s)

    def _flat_groups(self):
        ps = [p for g in self.param_groups for p in g["params"]]
        return _spaces(ps)

    def zero_grad(self, set_to_none: bool = False):
        spaces, loose = self._flat_groups()
        for sp, _ in spaces:
            sp.zero_grad()
        for p in loose:
            if p.grad is not None:
                if set_to_none:
                    p.grad = None
                else:
                    p.grad.zero_()

    def reset_state(self):
        """Zero every optimizer state buffer (K-AVG round boundary)."""
        from ..ops import kernels as K
        for bufs in self._state_bufs.values():
            for t in bufs.values():
                if t.is_cuda:
                    K.memset_(t)
                else:
                    t.zero_()
        self.state.clear()
        self._first = True
        self._step_host = 0
        for t in self._step_dev.values():
            t.zero_()
        for t in self._first_dev.values():
            t.fill_(1.0)

    def first_tensor(self, device):
        """fp32 device flag: 1 until the first fused step after a reset clears it."""
        t = self._first_dev.get(device)
        if t is None:
            t = torch.ones(1, dtype=torch.float32, device=device)
            self._first_dev[device] = t
        return t

    _STATE_NAMES = ()

    def begin_ranges(self):
        """Start of a step applied through ``step_range`` calls (no-op unless overridden)."""

    def prepare(self):
        """Allocate every device state buffer now (not lazily inside a first step), so
        :meth:`state_tensors` is complete before a graph capture."""
        spaces, _ = self._flat_groups()
        for sp, _ in spaces:
            if sp.device.type != "cuda":
                continue
            if self._STATE_NAMES:
                self._bufs(sp, list(self._STATE_NAMES))
            self.lr_tensor(sp.device)
            self.first_tensor(sp.device)
            self._step_dev.setdefault(sp.device, torch.zeros(1, dtype=torch.float32, device=sp.device))
        return self

    def state_tensors(self) -> List[torch.Tensor]:
        """Every device tensor :meth:`step` mutates."""
        out = [t for bufs in self._state_bufs.values() for t in bufs.values()]
        out += list(self._step_dev.values()) + list(self._first_dev.values())
        return out

    def _bufs(self, sp, names):
        key = id(sp)
        d = self._state_bufs.get(key)
        if d is None:
            d = {n: torch.zeros(sp.numel, dtype=torch.float32, device=sp.device) for n in names}
            self._state_bufs[key] = d
        return d


class SGD(FusedOptimizer):
    kind = "sgd"

    @property
    def _STATE_NAMES(self):
        return ("momentum",) if self.param_groups[0]["momentum"] != 0 else ()

    def __init__(self, params, lr=1e-3, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False):
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening,
                                      weight_decay=weight_decay, nesterov=nesterov))
        if len(self.param_groups) > 1:
            raise ValueError("fused SGD supports a single param group")

    def fuse_advance(self, ctr, batch, n) -> bool:
        """Can ``step(advance=(ctr, batch, n))`` advance the on-device data-sampler counter
        ``ctr`` (``ops.kernels.advance_counter_``) inside its SGD launch instead of a
        one-thread launch of its own?  False when no GPU flat space holds the counter's
        device.  Nothing is attached to the optimizer: the advance is per call."""
        spaces, _ = self._flat_groups()
        return bool(spaces and spaces[0][0].device.type == "cuda" and ctr.device == spaces[0][0].device)

    @torch.no_grad()
    def step(self, closure=None, advance=None):
        """advance: (ctr, batch, n) folded into this step's launch (see fuse_advance)."""
        loss = closure() if closure is not None else None
        g = self.param_groups[0]
        spaces, loose = self._flat_groups()
        for k, (sp, members) in enumerate(spaces):
            if sp.device.type != "cuda":
                loose += members
                continue
            sp.finish_grads()
            from ..ops import kernels as K
            mom = self._bufs(sp, ["momentum"])["momentum"] if g["momentum"] != 0 else None
            first = self.first_tensor(sp.device) if mom is not None else None
            K.sgd_(sp.master, sp.grad, mom, sp.shadow, g["lr"], wd=g["weight_decay"], momentum=g["momentum"],
                   dampening=g["dampening"], nesterov=g["nesterov"], first=self._first,
                   grad_scale=self._grad_scale, lr_dev=self.lr_tensor(sp.device), first_dev=first,
                   advance=advance if k == 0 else None)
            if first is not None:
                K.fill_(first, 0.0)
        if loose:
            _torch_sgd(loose, g, self.state, self._grad_scale)
        self._first = False
        return loss


    # ---- per-range steps (optimizer overlapped with backward, engine/dp.py) -------------
    def supports_ranges(self) -> bool:
        """True when every parameter lives in one flat space (no loose parameters)."""
        spaces, loose = self._flat_groups()
        return len(spaces) == 1 and not loose

    def supports_shard_range(self) -> bool:
        """One :meth:`step_range` per step over this rank's chunk (engine/dp.py shard plan)."""
        return self.supports_ranges()

    @torch.no_grad()
    def step_range(self, start: int, end: int, max_blocks: int = 0, advance_step: bool = True, advance=None):
        """The fused step restricted to flat elements [start, end): the gradients of a
        finished backward stage are applied while earlier stages still run backward.  The
        first-step flag stays set until :meth:`finish_ranges` (every range of the step
        reads the same value); the union of one step's ranges must cover the space once.
        advance_step: accepted for the ranged-step protocol (SGD keeps no step counter).
        advance: (ctr, batch, n) data-counter advance folded into this launch (as :meth:`step`)."""
        g = self.param_groups[0]
        spaces, loose = self._flat_groups()
        if len(spaces) != 1 or loose:
            raise ValueError("step_range needs all parameters in one flat space")
        sp = spaces[0][0]
        mom = self._bufs(sp, ["momentum"])["momentum"] if g["momentum"] != 0 else None
        if sp.device.type != "cuda":
            _sgd_range_cpu(sp, start, end, g, mom, self._first, self._grad_scale)
            return
        sp.finish_grads_range(start, end)
        from ..ops import kernels as K
        first = self.first_tensor(sp.device) if mom is not None else None
        K.sgd_(sp.master[start:end], sp.grad[start:end], None if mom is None else mom[start:end],
               None if sp.shadow is None else sp.shadow[start:end], g["lr"], wd=g["weight_decay"],
               momentum=g["momentum"], dampening=g["dampening"], nesterov=g["nesterov"], first=self._first,
               grad_scale=self._grad_scale, lr_dev=self.lr_tensor(sp.device), first_dev=first,
               max_blocks=max_blocks or _RANGE_BLOCKS, advance=advance)

    @torch.no_grad()
    def finish_ranges(self):
        """End of a step applied through :meth:`step_range`: clear the first-step flag."""
        spaces, _ = self._flat_groups()
        sp = spaces[0][0]
        if self.param_groups[0]["momentum"] != 0 and sp.device.type == "cuda":
            from ..ops import kernels as K
            K.fill_(self.first_tensor(sp.device), 0.0)
        self._first = False

# grid cap of a range update (it runs beside the backward on a side stream)
_RANGE_BLOCKS = 64


def _sgd_range_cpu(sp, start, end, g, mom, first, grad_scale):
    """torch form of k_sgd over [start, end) of a CPU flat space (same math as the kernel).
    Through ``.data``: parameters are views of the flat buffer and share its autograd version
    counter, which a range update must not bump while other stages' backward still runs."""
    w, gr = sp.master.data[start:end], sp.grad.data[start:end]
    d = gr * grad_scale if grad_scale != 1.0 else gr          # op for op as _torch_sgd
    if g["weight_decay"]:
        d = d.add(w, alpha=g["weight_decay"])
    if mom is not None:
        m = mom.data[start:end]
        if first:
            m.copy_(d)
        else:
            m.mul_(g["momentum"]).add_(d, alpha=1 - g["dampening"])
        d = d.add(m, alpha=g["momentum"]) if g["nesterov"] else m
    w.add_(d, alpha=-g["lr"])
    if sp.shadow is not None:
        sp.shadow.data[start:end].copy_(w)


def _torch_sgd(params, g, state, grad_scale):
    for p in params:
        if p.grad is None:
            continue
        d = p.grad * grad_scale if grad_scale != 1.0 else p.grad
        if g["weight_decay"]:
            d = d.add(p, alpha=g["weight_decay"])
        if g["momentum"]:
            st = state.setdefault(p, {})
            buf = st.get("momentum_buffer")
            if buf is None:
                buf = d.clone().detach()
                st["momentum_buffer"] = buf
            else:
                buf.mul_(g["momentum"]).add_(d, alpha=1 - g["dampening"])
            d = d.add(buf, alpha=g["momentum"]) if g["nesterov"] else buf
        p.add_(d, alpha=-g["lr"])


class Adam(FusedOptimizer):
    kind = "adam"
    decoupled = False
    _STATE_NAMES = ("exp_avg", "exp_avg_sq")

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        if len(self.param_groups) > 1:
            raise ValueError("fused Adam supports a single param group")

    def step_tensor(self, device):
        t = self._step_dev.get(device)
        if t is None:
            t = torch.zeros(1, dtype=torch.float32, device=device)
            self._step_dev[device] = t
        return t

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        spaces, loose = self._flat_groups()
        self._step_host += 1
        for sp, members in spaces:
            if sp.device.type != "cuda":
                loose += members
                continue
            sp.finish_grads()
            from ..ops import kernels as K
            st = self._step_dev_inc(sp.device)
            bufs = self._bufs(sp, ["exp_avg", "exp_avg_sq"])
            K.adam_(sp.master, sp.grad, bufs["exp_avg"], bufs["exp_avg_sq"], sp.shadow, g["lr"], 0.0, b1, b2,
                    g["eps"], g["weight_decay"], self.decoupled, self._grad_scale,
                    lr_dev=self.lr_tensor(sp.device), step_dev=st)
        if loose:
            _torch_adam(loose, g, self.state, self._grad_scale, self.decoupled)
        return loss

    def supports_ranges(self) -> bool:
        """Per-backward-stage updates (engine/dp.py ``opt_overlap``): :meth:`begin_ranges`
        advances the bias-correction step once, then every stage's :meth:`step_range` runs with
        ``advance_step=False``, so a step split into ranges equals one whole step."""
        spaces, loose = self._flat_groups()
        return len(spaces) == 1 and not loose and spaces[0][0].device.type == "cuda"

    @torch.no_grad()
    def begin_ranges(self):
        """Start of a step applied as several ranges: advance the step counter once."""
        spaces, _ = self._flat_groups()
        self._step_host += 1
        self._step_dev_inc(spaces[0][0].device)

    def finish_ranges(self):
        """End of a ranged step (nothing to clear: the counter advanced in begin_ranges)."""

    def supports_shard_range(self) -> bool:
        """One :meth:`step_range` per step over this rank's chunk (engine/dp.py shard plan)."""
        spaces, loose = self._flat_groups()
        return len(spaces) == 1 and not loose and spaces[0][0].device.type == "cuda"

    @torch.no_grad()
    def step_range(self, start: int, end: int, max_blocks: int = 0, advance_step: bool = True):
        """The fused step over flat elements [start, end) only.  advance_step=True (a sharded
        update: this rank owns that chunk of the master and its moments, one range per step)
        advances the step counter; False (one of several stage ranges of a step, after
        :meth:`begin_ranges`) reuses it."""
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        spaces, loose = self._flat_groups()
        if len(spaces) != 1 or loose:
            raise ValueError("step_range needs all parameters in one flat space")
        sp = spaces[0][0]
        from ..ops import kernels as K
        if advance_step:
            self._step_host += 1
            st = self._step_dev_inc(sp.device)
        else:
            st = self.step_tensor(sp.device)
        sp.finish_grads_range(start, end)
        bufs = self._bufs(sp, ["exp_avg", "exp_avg_sq"])
        if end > start:
            K.adam_(sp.master[start:end], sp.grad[start:end], bufs["exp_avg"][start:end],
                    bufs["exp_avg_sq"][start:end], None if sp.shadow is None else sp.shadow[start:end], g["lr"], 0.0,
                    b1, b2, g["eps"], g["weight_decay"], self.decoupled, self._grad_scale,
                    lr_dev=self.lr_tensor(sp.device), step_dev=st,
                    max_blocks=max_blocks or (0 if advance_step else _RANGE_BLOCKS))

    def _step_dev_inc(self, device):
        from ..ops import kernels as K
        t = self.step_tensor(device)
        K.increment_(t, 1.0)
        return t


class AdamW(Adam):
    kind = "adamw"
    decoupled = True

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        super().__init__(params, lr, betas, eps, weight_decay)


def _torch_adam(params, g, state, grad_scale, decoupled):
    b1, b2 = g["betas"]
    for p in params:
        if p.grad is None:
            continue
        st = state.setdefault(p, {})
        if not st:
            st["step"] = 0
            st["exp_avg"] = torch.zeros_like(p)
            st["exp_avg_sq"] = torch.zeros_like(p)
        st["step"] += 1
        t = st["step"]
        gr = p.grad * grad_scale
        if decoupled:
            p.mul_(1 - g["lr"] * g["weight_decay"])
        elif g["weight_decay"]:
            gr = gr.add(p, alpha=g["weight_decay"])
        st["exp_avg"].mul_(b1).add_(gr, alpha=1 - b1)
        st["exp_avg_sq"].mul_(b2).addcmul_(gr, gr, value=1 - b2)
        bc1 = 1 - b1 ** t
        bc2 = 1 - b2 ** t
        denom = (st["exp_avg_sq"].sqrt() / (bc2 ** 0.5)).add_(g["eps"])
        p.addcdiv_(st["exp_avg"], denom, value=-g["lr"] / bc1)


def from_torch(opt: torch.optim.Optimizer) -> FusedOptimizer:
    """Fused equivalent of a stock torch optimizer (same params and hyper-parameters)."""
    if isinstance(opt, FusedOptimizer):
        return opt
    params = [p for g in opt.param_groups for p in g["params"]]
    g = opt.param_groups[0]
    if isinstance(opt, torch.optim.AdamW):
        return AdamW(params, lr=g["lr"], betas=g["betas"], eps=g["eps"], weight_decay=g["weight_decay"])
    if isinstance(opt, torch.optim.Adam):
        return Adam(params, lr=g["lr"], betas=g["betas"], eps=g["eps"], weight_decay=g["weight_decay"])
    if isinstance(opt, torch.optim.SGD):
        return SGD(params, lr=g["lr"], momentum=g["momentum"], dampening=g["dampening"],
                   weight_decay=g["weight_decay"], nesterov=g["nesterov"])
    raise TypeError(f"no fused equivalent for {type(opt).__name__}")
