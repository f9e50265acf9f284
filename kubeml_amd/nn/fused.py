"""Fused conv -> BatchNorm -> (+residual) -> ReLU units and block-level autograd.

A ``ConvBNUnit`` is the basic building block of the CNN workloads (ResNet-34/50,
VGG-16-BN).  Its training forward is two kernels:

    conv_igemm (FWD, epilogue accumulates per-channel sum/sumsq)  ->  bn_apply(+res, ReLU)

and its backward three:

    bn_bwd (reduce + apply, ReLU mask, residual-gradient copy)  ->  conv WGRAD (split-K,
    into the flat fp32 grad buffer)  ->  conv DGRAD (epilogue adds the other branch's
    input gradient, so residual merges cost no separate add kernel).

Whole residual blocks are single autograd nodes (``BlockFn``) so PyTorch's autograd
never inserts its own gradient-accumulation kernels between our launches: the
entire step runs on the HIP kernels and captures cleanly into one hipGraph.

BN statistics travel as per-wave partial rows from the conv epilogue to bn_apply (plain
stores, summed in a fixed order: no zeroing, no atomics, deterministic).
"""
from __future__ import annotations

from typing import List, Optional

import torch
from torch.autograd import Function

import os

from .flat import grad_out, grad_out_pair, master_of, shadow_of

# every BN backward takes its dgamma/dbeta partial rows from the dgrad epilogue that produced
# its input gradient (False: its own reduction pass; tests compare the two).  Folding the BN
# backward into the next conv pair's dz staging measured 1.3-2.6x slower pairs even with the rows
# pre-reduced to one (profiles/r5/bn_fold_ab.md, profiles/r6/bn_final_rows.md): removed.
_BN_FUSE = True


def _wg_buf(conv, x):
    """Persistent [4K,1,1,4C] fp32 scratch of an unrolled conv's 1x1-form weight gradient
    (stable address: graphs), folded onto the 3x3 taps by the flat space (defer_fold22)."""
    Kc, _, _, C = conv.weight._kml_grad_storage.shape
    shape = (4 * Kc, 1, 1, 4 * C)
    buf = getattr(conv, "_kml_wg_buf", None)
    if buf is None or tuple(buf.shape) != shape or buf.device != x.device:
        buf = torch.empty(shape, dtype=torch.float32, device=x.device)
        object.__setattr__(conv, "_kml_wg_buf", buf)
    return buf


def _wgrad_target(conv, x, unroll):
    """(weight-gradient destination, accumulate) — the 1x1-form scratch for an unrolled conv."""
    if unroll:
        return _wg_buf(conv, x), False
    return grad_out(conv.weight)


def _wgrad(x, dc, conv, unroll=False, rider=None):
    from ..ops import kernels as K
    kh, kw = conv.kernel_size
    dw, acc = _wgrad_target(conv, x, unroll)
    K.conv_wgrad(x, dc, dw, kh, kw, conv.stride, conv.padding, unroll=unroll, accumulate=acc, rider=rider)
    if unroll:
        conv.weight._kml_flat.defer_fold22(conv.weight, dw)


def _wu_buf(conv, w):
    """Persistent [4K,1,1,4C] buffer of a conv's unrolled weight (stable address: graphs)."""
    Kc, _, _, C = w.shape
    shape = (4 * Kc, 1, 1, 4 * C)
    buf = getattr(conv, "_kml_wu_buf", None)
    if buf is None or tuple(buf.shape) != shape or buf.device != w.device:
        buf = torch.empty(shape, dtype=torch.bfloat16, device=w.device)
        object.__setattr__(conv, "_kml_wu_buf", buf)
    return buf


def unrolled_for(conv, x):
    """Unrolled weight for this training forward of ``conv`` on ``x`` (ops.kernels.unrolled22),
    or None when the conv runs in its ordinary form.  Uses the copy refresh_transposed made
    at the start of this forward, else gathers it now (and marks the conv for batching);
    kept on the module for this forward's backward."""
    from ..ops import kernels as K
    if not x.is_cuda:
        return None
    kh, kw = conv.kernel_size
    if not K.unrolled22(x.shape[1], x.shape[2], kh, kw, conv.stride, conv.padding):
        return None
    w = shadow_of(conv.weight)
    if _U22_GATHER and w.shape[3] % 8 == 0 and K.bwd_plans(
            x.shape, w.shape[0], kh, kw, conv.stride, conv.padding, unroll=True)[0][4] != K.DIRECT:
        # the kernels gather the unrolled weight from w: no copy to make or keep fresh
        object.__setattr__(conv, "_kml_wu", K.GATHER22)
        return K.GATHER22
    buf = _wu_buf(conv, w)
    if not getattr(conv, "_kml_wu_fresh", False):
        object.__setattr__(conv, "_kml_wants_wu", True)
        K.unroll22_multi([w], [buf])
    object.__setattr__(conv, "_kml_wu_fresh", False)   # one forward per refresh
    object.__setattr__(conv, "_kml_wu", buf)           # for this forward's backward
    return buf


_U22_GATHER = True    # unrolled 2x2 convs read the 3x3 weight through a gather (no materialised copy)


def refresh_transposed(convs):
    """Derived bf16 weights of this training step, each kind in ONE launch per 16 convs,
    at the start of a training forward:

    * unrolled weights ``[4K,1,1,4C]`` of the convs that run in the dense 2x2-map form
      (:func:`unrolled_for`, ops.kernels.unrolled22);
    * transposed weights ``[Cin][KH][KW][Kp]`` for every conv whose dgrad runs the direct
      (LDS-free) variant (of the unrolled weight for an unrolled conv).

    Which convs need them is learned from earlier passes (the forward / backward mark
    them); a conv not yet marked makes its copy inline.  A transposed copy is consumed
    (and dropped) by that conv's next backward."""
    from ..ops import kernels as K
    unr = [c for c in convs if getattr(c, "_kml_wants_wu", False)]
    ws, wus = [], []
    for c in unr:
        w = shadow_of(c.weight)
        ws.append(w)
        wus.append(_wu_buf(c, w))
        object.__setattr__(c, "_kml_wu_fresh", True)
    for i in range(0, len(ws), 16):
        K.unroll22_multi(ws[i:i + 16], wus[i:i + 16])
    want = [c for c in convs if getattr(c, "_kml_wants_wt", False)]
    ws, wts = [], []
    for c in want:
        w = c._kml_wu_buf if getattr(c, "_kml_wants_wu", False) else shadow_of(c.weight)
        Kc, KH, KW, C = w.shape
        shape = (C, KH, KW, -(-Kc // 32) * 32)
        buf = getattr(c, "_kml_wt_buf", None)
        if buf is None or tuple(buf.shape) != shape or buf.device != w.device:
            buf = torch.empty(shape, dtype=torch.bfloat16, device=w.device)
            object.__setattr__(c, "_kml_wt_buf", buf)
        ws.append(w)
        wts.append(buf)
        object.__setattr__(c, "_kml_wt", buf)
    for i in range(0, len(ws), 16):
        K.weight_transpose_multi(ws[i:i + 16], wts[i:i + 16])


class BNRegistry:
    """The BatchNorm layers of a model in forward order (used for the packed
    ``num_batches_tracked`` counters).  BN statistics need no arena: the conv epilogue
    writes per-wave partial rows into a fresh buffer that bn_apply sums (every row is
    written, so nothing is zeroed per step)."""

    def __init__(self, bns):
        self.bns = list(bns)


# bn1 + ReLU of a BasicBlock folded into conv2's halo patch staging (BlockFn.forward); False:
# every BatchNorm runs its own apply kernel (tests compare the two)
_BN_FOLD = True
# group-reduce the folded BN's statistics rows in the producing conv (<= 16 rows for the consumer);
# off: measured slower (1.354 vs 1.333 ms/step) and the ungrouped fold is bit-identical to the
# unfolded BN apply (tests/test_models_gpu.py::test_resnet34_bn_fold_matches_unfolded)
_FOLD_GROUP = False


def _conv_bias(conv):
    """fp32 storage of a conv's bias (VGG), or None.

    Its gradient is never produced: in front of a training-mode BatchNorm a per-channel bias
    has an identically zero gradient — the BN backward output dc = a (dy - mean(dy) - xhat
    mean(dy xhat)) sums to a (sum dy - sum dy - mean(dy xhat) sum xhat) = 0 per channel because
    sum xhat = 0 — so the region stays zero (FlatParamSpace.finish_grads zeroes regions nobody
    wrote) instead of column-summing rounding noise.  The forward still adds it, so batch and
    running statistics (and eval outputs, checkpoints) match torch's conv(+bias) -> BN."""
    b = getattr(conv, "bias", None)
    return master_of(b) if b is not None else None


class ConvBNUnit:
    """Stateless executor for (conv module, bn module, relu)."""

    @staticmethod
    def conv_rows(x, conv, group=False):
        """Training conv with per-tile BN partial statistics rows (no BN applied):
        (c, rows, G).  group: reduce the rows to <= 16 in the producing launch (for a
        consumer whose every block sums them: the BN-folding halo conv)."""
        from ..ops import kernels as K
        w = shadow_of(conv.weight)
        kh, kw = conv.kernel_size
        K_out = w.shape[0]
        wu = unrolled_for(conv, x) if _conv_bias(conv) is None else None
        if wu is not None:    # the unrolled 1x1 form writes folded rows (never group-reduced)
            G = K.conv_fwd_stats_rows(x.shape, K_out, kh, kw, conv.stride, conv.padding, unroll=True)
            stats = torch.empty(G * 2 * K_out, dtype=torch.float32, device=x.device)
            c = K.conv_fwd(x, w, kh, kw, conv.stride, conv.padding, stats=stats, stats_part=True, wu=wu)
            return c, stats, G
        G = K.conv_fwd_stats_rows(x.shape, K_out, kh, kw, conv.stride, conv.padding, group=group)
        stats = torch.empty(G * 2 * K_out, dtype=torch.float32, device=x.device)
        c = K.conv_fwd(x, w, kh, kw, conv.stride, conv.padding, bias=_conv_bias(conv), stats=stats, stats_part=True,
                       stats_group=group)
        return c, stats, G

    @staticmethod
    def forward_folded(c_in, rows_in, G_in, bn_in, x_in, conv, bn, relu: bool, res: Optional[torch.Tensor],
                       defer: bool = False):
        """conv(relu(bn_in(c_in))) with bn_in applied inside the conv's patch staging
        (ops.kernels.conv_fwd_bnin), then this unit's own BN.  Returns (y, saved of the bn_in
        unit, saved of this unit).  defer: this unit's BN is NOT applied — y, mean and rstd are
        empty buffers that the next block's first conv fills (:class:`PendingBN`), returned as the
        4th element."""
        from ..ops import kernels as K
        C = c_in.shape[-1]
        y_in = torch.empty_like(c_in)
        mean_in = torch.empty(C, dtype=torch.float32, device=c_in.device)
        rstd_in = torch.empty_like(mean_in)
        w = shadow_of(conv.weight)
        K_out = w.shape[0]
        unrolled_for(conv, c_in)      # marks this forward's form (unrolled 2x2: GATHER22) for the backward
        G = K.bnin_stats_rows(c_in.shape, K_out)
        stats = torch.empty(G * 2 * K_out, dtype=torch.float32, device=c_in.device)
        c = K.conv_fwd_bnin(c_in, w, rows_in, G_in, master_of(bn_in.weight), master_of(bn_in.bias), mean_in, rstd_in,
                            bn_in.running_mean, bn_in.running_var, bn_in.eps,
                            bn_in.momentum if bn_in.momentum is not None else 0.1, y_in, stats=stats, stats_part=True)
        mean = torch.empty(K_out, dtype=torch.float32, device=c_in.device)
        rstd = torch.empty_like(mean)
        if defer:
            y = torch.empty_like(c)
            pend = PendingBN(y, c, stats, G, bn, res, mean, rstd, relu)
            return y, (x_in, c_in, y_in, mean_in, rstd_in), (y_in, c, y if relu else None, mean, rstd), pend
        y = K.bn_apply(c, stats, master_of(bn.weight), master_of(bn.bias), res=res, save_mean=mean, save_rstd=rstd,
                       run_mean=bn.running_mean, run_var=bn.running_var, eps=bn.eps,
                       momentum=bn.momentum if bn.momentum is not None else 0.1, relu=relu, stats_rows=G)
        return y, (x_in, c_in, y_in, mean_in, rstd_in), (y_in, c, y if relu else None, mean, rstd)

    @staticmethod
    def conv_rows_pending(pend, h, conv):
        """conv_rows(h, conv) where h is the EMPTY output of the previous block (``pend``): the
        previous block's last BN (+ residual + ReLU) is applied while this conv stages its input
        (ops.kernels.conv_fwd_bnin with res), which also writes h, the BN's saved mean / rstd and
        its running statistics.  Returns (c, rows, G) like conv_rows."""
        from ..ops import kernels as K
        bn = pend.bn
        w = shadow_of(conv.weight)
        K_out = w.shape[0]
        unrolled_for(conv, h)         # this forward's form of conv (unrolled 2x2: GATHER22) for the backward
        G = K.bnin_stats_rows(h.shape, K_out)
        stats = torch.empty(G * 2 * K_out, dtype=torch.float32, device=h.device)
        c = K.conv_fwd_bnin(pend.c, w, pend.rows, pend.G, master_of(bn.weight), master_of(bn.bias), pend.mean,
                            pend.rstd, bn.running_mean, bn.running_var, bn.eps,
                            bn.momentum if bn.momentum is not None else 0.1, h, stats=stats, stats_part=True,
                            res=pend.res)
        return c, stats, G

    @staticmethod
    def conv_stats(x, conv):
        """The training conv of :meth:`forward`: (c, stats rows, G).  Per-wave partial statistics
        from the conv epilogue (plain stores, every row written: no zeroing, no atomics); the BN
        apply sums them in its prologue."""
        from ..ops import kernels as K
        w = shadow_of(conv.weight)
        kh, kw = conv.kernel_size
        bias = _conv_bias(conv)
        K_out = w.shape[0]
        wu = unrolled_for(conv, x) if bias is None else None   # the 1x1 form has no bias epilogue
        G = K.conv_fwd_stats_rows(x.shape, K_out, kh, kw, conv.stride, conv.padding, unroll=wu is not None)
        stats = torch.empty(G * 2 * K_out, dtype=torch.float32, device=x.device)
        c = K.conv_fwd(x, w, kh, kw, conv.stride, conv.padding, bias=bias, stats=stats, stats_part=True, wu=wu)
        return c, stats, G

    @staticmethod
    def bn_train(c, stats, G, x, bn, relu: bool, res: Optional[torch.Tensor]):
        """The training BN of :meth:`forward` over the conv output ``c`` of input ``x``."""
        from ..ops import kernels as K
        C = c.shape[-1]
        mean = torch.empty(C, dtype=torch.float32, device=c.device)
        rstd = torch.empty_like(mean)
        y = K.bn_apply(c, stats, master_of(bn.weight), master_of(bn.bias), res=res, save_mean=mean, save_rstd=rstd,
                       run_mean=bn.running_mean, run_var=bn.running_var, eps=bn.eps,
                       momentum=bn.momentum if bn.momentum is not None else 0.1, relu=relu, stats_rows=G)
        return y, (x, c, y if relu else None, mean, rstd)

    @staticmethod
    def forward(x, conv, bn, relu: bool, res: Optional[torch.Tensor], training: bool):
        from ..ops import kernels as K
        if training:
            c, stats, G = ConvBNUnit.conv_stats(x, conv)
            return ConvBNUnit.bn_train(c, stats, G, x, bn, relu, res)
        w = shadow_of(conv.weight)
        kh, kw = conv.kernel_size
        gamma, beta = master_of(bn.weight), master_of(bn.bias)
        bias = _conv_bias(conv)
        c = K.conv_fwd(x, w, kh, kw, conv.stride, conv.padding, bias=bias)
        y = K.bn_apply(c, None, gamma, beta, res=res, run_mean=bn.running_mean, run_var=bn.running_var,
                       eps=bn.eps, relu=relu, training=False)
        return y, None

    @staticmethod
    def backward(dy, saved, conv, bn, want_dres: bool, need_dx: bool, addend=None, partial=None, consumer=None):
        """BN backward -> conv wgrad -> conv dgrad.  ``partial``: this BN's dgamma/dbeta
        partial rows, already produced by the dgrad that computed ``dy`` — that dgrad also
        applied this BN's ReLU mask (``bnf_mask``), so ``dy`` is already dz: the BN backward
        skips the reduction pass and never reads y.  ``consumer``: saved state
        (x, c, y, mean, rstd) of the BN that will consume dx — its partial rows are produced
        here, its mask applied to dx, and the partials returned."""
        dc, dres, wu = ConvBNUnit.bn_backward(dy, saved, conv, bn, want_dres, partial)
        dx, part_out = ConvBNUnit.conv_backward(dc, saved, conv, need_dx, wu, addend, consumer)
        return dx, dres, part_out

    @staticmethod
    def bn_backward(dy, saved, conv, bn, want_dres: bool, partial=None):
        """The BN half of :meth:`backward`: (dc, dres, the conv's unrolled-form marker)."""
        from ..ops import kernels as K
        x, c, y, mean, rstd = saved
        dg, db, acc = grad_out_pair(bn.weight, bn.bias)
        wu = getattr(conv, "_kml_wu", None) if x.is_cuda else None   # set by this step's forward
        dres = torch.empty_like(dy) if want_dres else None
        dc = K.bn_bwd(dy, None if partial is not None else y, c, mean, rstd, master_of(bn.weight),
                      dg, db, dres=dres, partial=partial, accumulate=acc, rider=_take_rider(bn))
        object.__setattr__(conv, "_kml_wu", None)
        return dc, dres, wu

    @staticmethod
    def conv_backward(dc, saved, conv, need_dx: bool, wu, addend=None, consumer=None):
        """The conv half of :meth:`backward`: (dx, consumer partial rows)."""
        from ..ops import kernels as K
        x = saved[0]
        kh, kw = conv.kernel_size
        dx, part_out = None, None
        bnf = None if consumer is None else (consumer[2], consumer[1], consumer[3], consumer[4])
        if need_dx:
            # dgrad + wgrad as one grouped launch (falls back to two for unpaired plans)
            w = shadow_of(conv.weight)
            wt = getattr(conv, "_kml_wt", None)
            if wt is None and K.bwd_plans(x.shape, w.shape[0], kh, kw, conv.stride, conv.padding,
                                          unroll=wu is not None)[0][4] == K.DIRECT:
                object.__setattr__(conv, "_kml_wants_wt", True)   # batched by refresh_transposed()
            dw, acc = _wgrad_target(conv, x, wu is not None)
            r = K.conv_bwd(dc, w, x, dw, kh, kw, conv.stride, conv.padding,
                           addend=addend, bnf=bnf, wt=wt, wu=wu, bnf_mask=True, accumulate=acc,
                           rider=_take_rider(conv))
            if wu is not None:
                conv.weight._kml_flat.defer_fold22(conv.weight, dw)
            object.__setattr__(conv, "_kml_wt", None)             # valid for one backward pass
            dx, part_out = r if bnf is not None else (r, None)
            return dx, part_out
        _wgrad(x, dc, conv, unroll=wu is not None, rider=_take_rider(conv))
        if need_dx:
            r = K.conv_dgrad(dc, shadow_of(conv.weight), x.shape, kh, kw, conv.stride, conv.padding,
                             addend=addend, bnf=bnf, wu=wu, bnf_mask=True)
            dx, part_out = r if bnf is not None else (r, None)
        return dx, part_out


def _take_rider(conv):
    """The optimizer-update rider armed on this conv for the current backward (engine/dp.py
    ``ride``: a callable returning an ``ops.kernels.SgdRider`` or None), else None."""
    r = getattr(conv, "_kml_rider", None)
    return r() if r is not None else None


class PendingBN:
    """A residual block's output BN (+ residual + ReLU) left unapplied for the next block's first
    conv to apply while staging its input (cross-block fold, :func:`_defer_target`).  ``y`` is
    the block output buffer, still empty; :meth:`materialize` is the fallback (one BN apply)."""
    __slots__ = ("y", "c", "rows", "G", "bn", "res", "mean", "rstd", "relu")

    def __init__(self, y, c, rows, G, bn, res, mean, rstd, relu):
        self.y, self.c, self.rows, self.G, self.bn = y, c, rows, G, bn
        self.res, self.mean, self.rstd, self.relu = res, mean, rstd, relu

    def materialize(self):
        from ..ops import kernels as K
        bn = self.bn
        K.bn_apply(self.c, self.rows, master_of(bn.weight), master_of(bn.bias), y=self.y, res=self.res,
                   save_mean=self.mean, save_rstd=self.rstd, run_mean=bn.running_mean, run_var=bn.running_var,
                   eps=bn.eps, momentum=bn.momentum if bn.momentum is not None else 0.1, relu=self.relu,
                   stats_rows=self.G)


# cross-block fold: a BasicBlock's output BN + residual + ReLU is applied by the next block's first
# conv (halo / one-shot BN-in staging) instead of its own launch.  Only inside a model forward that
# drives the chain (``chain()``: ResNet.forward), so a block called on its own never defers.
_CROSS_FOLD = True
_CHAIN = [0]


class chain:
    """Context of a model forward whose blocks may defer their output BN to the next block."""

    def __init__(self, blocks):
        self.blocks = blocks

    def __enter__(self):
        _CHAIN[0] += 1
        return self

    def __exit__(self, *exc):
        _CHAIN[0] -= 1
        for b in self.blocks:   # safety: a deferred output nobody consumed is applied here
            pend = getattr(b, "_kml_pend_in", None)
            if pend is not None:
                object.__setattr__(b, "_kml_pend_in", None)
                pend.materialize()
        return False


def _defer_target(block, out_shape):
    """The next block if it will apply this block's output BN in its first conv, else None."""
    if not (_CROSS_FOLD and _BN_FOLD and _CHAIN[0] > 0):
        return None
    ref = getattr(block, "_kml_next_ref", None)
    nxt = ref() if ref is not None else None
    if nxt is None or not nxt.training or any(u[3] == "short" for u in nxt._kml_plan):
        return None
    from ..ops import kernels as K
    if _fold_unit_shape(out_shape, nxt._kml_plan) is None:
        return None
    conv1 = nxt._kml_plan[0][0]
    if conv1.kernel_size != (3, 3) or tuple(conv1.stride) != (1, 1) or tuple(conv1.padding) != (1, 1):
        return None
    return nxt if K.bnin_ok(out_shape, shadow_of(conv1.weight).shape[0], 3, 3, (1, 1), (1, 1)) else None


class BlockFn(Function):
    """Autograd node for a residual block described by a ``plan`` of units.

    plan: list of (conv, bn, relu, role) in forward order where role is one of
      "main"   — unit on the main branch fed by the previous main output
      "short"  — projection shortcut fed by the block input
      "last"   — final main unit; its BN adds the shortcut (identity or "short")
    """

    @staticmethod
    def forward(ctx, x, block, *params):
        training = True
        plan = block._kml_plan
        saved = [None] * len(plan)
        fold = _fold_unit(x, plan)      # index of a main unit whose BN + ReLU the next conv applies
        # the previous block's output BN, deferred to this block's first conv (x is still empty)
        pend_in = getattr(block, "_kml_pend_in", None)
        object.__setattr__(block, "_kml_pend_in", None)
        if pend_in is not None and (pend_in.y.data_ptr() != x.data_ptr() or fold != 0):
            pend_in.materialize()
            pend_in = None
        h = x
        short = None
        pending = None
        pre = {}
        done = set()   # units of pre whose BN is already applied: (y, saved)
        if _FWD_PAIR and pend_in is None and len(plan) > 2 and plan[0][3] == "main" and plan[1][3] == "short" \
                and x.is_cuda:
            # a downsampling block: its first conv and the projection both read x — one launch
            # (ops.kernels.conv_fwd_pair) when their plans pair; both BN applies follow
            from ..ops import kernels as K
            with K.conv_fwd_pair():
                pre[0] = (ConvBNUnit.conv_rows(x, plan[0][0], group=_FOLD_GROUP) if fold == 0
                          else ConvBNUnit.conv_stats(x, plan[0][0]))
                pre[1] = ConvBNUnit.conv_stats(x, plan[1][0])
            if fold != 0:   # both BN applies in one launch as well (bn_apply_pair)
                with K.bn_apply_pair():
                    pre[0] = ConvBNUnit.bn_train(*pre[0], x, plan[0][1], plan[0][2], None)
                    pre[1] = ConvBNUnit.bn_train(*pre[1], x, plan[1][1], plan[1][2], None)
                done = {0, 1}
        for i, (conv, bn, relu, role) in enumerate(plan):
            if role == "short":
                if i in done:
                    short, saved[i] = pre[i]
                elif i in pre:
                    short, saved[i] = ConvBNUnit.bn_train(*pre[i], x, bn, relu, None)
                else:
                    short, saved[i] = ConvBNUnit.forward(x, conv, bn, relu, None, training)
            elif i == fold:
                if pend_in is not None:
                    c, rows, G = ConvBNUnit.conv_rows_pending(pend_in, h, conv)
                    pend_in = None
                elif i in pre:
                    c, rows, G = pre[i]
                else:
                    c, rows, G = ConvBNUnit.conv_rows(h, conv, group=_FOLD_GROUP)
                pending = (i, h, c, rows, G, bn)
            elif pending is not None:   # the conv right after the folded unit ("last": + residual)
                j, x_in, c_in, rows, G, bn_in = pending
                res = (short if short is not None else x) if role == "last" else None
                nxt = _defer_target(block, (x.shape[0],) + _out_hw_c(c_in.shape, conv)) if role == "last" else None
                r = ConvBNUnit.forward_folded(c_in, rows, G, bn_in, x_in, conv, bn, relu, res, defer=nxt is not None)
                h, saved[j], saved[i] = r[:3]
                if nxt is not None:
                    object.__setattr__(nxt, "_kml_pend_in", r[3])
                pending = None
            elif role == "last":
                res = short if short is not None else x
                h, saved[i] = ConvBNUnit.forward(h, conv, bn, relu, res, training)
            elif i in done:
                h, saved[i] = pre[i]
            elif i in pre:
                h, saved[i] = ConvBNUnit.bn_train(*pre[i], h, bn, relu, None)
            else:
                h, saved[i] = ConvBNUnit.forward(h, conv, bn, relu, None, training)
        ctx.block = block
        ctx.saved = saved
        # the next block's first dgrad produces this block's output gradient; it can emit
        # the dgamma/dbeta partials of our last BN if it can see that BN's saved state
        last = [i for i, u in enumerate(block._kml_plan) if u[3] == "last"]
        object.__setattr__(block, "_kml_last_saved", saved[last[0]] if last else None)
        object.__setattr__(block, "_kml_in_partial", None)
        return h

    @staticmethod
    def backward(ctx, dout):
        block = ctx.block
        plan = block._kml_plan
        saved = ctx.saved
        dout = dout.contiguous()
        need_x = ctx.needs_input_grad[0]
        # partials of our last BN computed by the next block's first dgrad (same tensor only)
        stash = getattr(block, "_kml_in_partial", None)
        in_partial = stash[1] if stash is not None and stash[0] == dout.data_ptr() else None
        object.__setattr__(block, "_kml_in_partial", None)
        prev_ref = getattr(block, "_kml_prev_ref", None)
        prev = prev_ref() if prev_ref is not None else None
        prev_saved = getattr(prev, "_kml_last_saved", None) if prev is not None else None
        # walk main units backwards; the last unit also yields the shortcut gradient dz
        main = [(i, u) for i, u in enumerate(plan) if u[3] != "short"]
        short = [(i, u) for i, u in enumerate(plan) if u[3] == "short"]
        g = dout
        dres = None
        partial = in_partial
        for k in range(len(main) - 1, -1, -1):
            i, (conv, bn, relu, role) = main[k]
            is_last = role == "last"
            is_first = k == 0
            addend = None
            swap = is_first and short and not is_last and _short_last(saved[short[0][0]], short[0][1][0], conv)
            consumer = saved[main[k - 1][0]] if k > 0 else (prev_saved if need_x else None)
            if not _BN_FUSE:
                consumer = None
            if is_first and not swap and short and not is_last and _BWD_PAIR and dout.is_cuda:
                # the projection's BN backward and this unit's are independent: one apply launch
                # (ops.kernels.bn_bwd_pair), then the projection's conv backward (its dgrad is this
                # unit's dgrad addend), then this unit's
                from ..ops import kernels as K
                j, (sc, sb, _, _) = short[0]
                with K.bn_bwd_pair():
                    dc_s, _, wu_s = ConvBNUnit.bn_backward(dres, saved[j], sc, sb, False)
                    dc, _, wu = ConvBNUnit.bn_backward(g, saved[i], conv, bn, False, partial)
                addend, _ = ConvBNUnit.conv_backward(dc_s, saved[j], sc, need_x, wu_s)
                g, partial = ConvBNUnit.conv_backward(dc, saved[i], conv, need_x, wu, addend, consumer)
                continue
            if is_first and not swap:
                # shortcut gradient joins here: identity -> dres, projection -> its dgrad
                if short:
                    j, (sc, sb, sr, _) = short[0]
                    addend, _, _ = ConvBNUnit.backward(dres, saved[j], sc, sb, False, need_x)
                else:
                    addend = dres
            if swap:
                # strided projection shortcut on a large map: the main conv's dgrad runs plain and the
                # shortcut's dgrad takes it as its residual addend plus the consumer-BN epilogue —
                # with operands, the stride-2 dgrad runs by parity class (3/4 of its output rows are
                # epilogue only) instead of multiplying the zero taps of the whole input map
                j, (sc, sb, _, _) = short[0]
                dx1, _, _ = ConvBNUnit.backward(g, saved[i], conv, bn, want_dres=False, need_dx=need_x,
                                                partial=partial)
                g, _, partial = ConvBNUnit.backward(dres, saved[j], sc, sb, False, need_x, addend=dx1,
                                                    consumer=consumer)
                continue
            dx, dz, part_out = ConvBNUnit.backward(g, saved[i], conv, bn, want_dres=is_last,
                                                   need_dx=(not is_first) or need_x,
                                                   addend=addend if is_first else None, partial=partial,
                                                   consumer=consumer)
            if is_last:
                dres = dz
            g = dx
            partial = part_out
        if prev is not None and partial is not None and g is not None:
            object.__setattr__(prev, "_kml_in_partial", (g.data_ptr(), partial))
        ctx.saved = None
        object.__setattr__(block, "_kml_last_saved", None)
        return (g, None) + (None,) * (len(ctx.needs_input_grad) - 2)


_SHORT_LAST = True
# downsampling blocks launch their first conv and the projection as one forward pair, and their
# two BN backward applies as one launch (same switch)
_FWD_PAIR = os.environ.get("KUBEML_FWD_PAIR", "1") != "0"
_BWD_PAIR = _FWD_PAIR


def _short_last(short_saved, sc, conv1) -> bool:
    """Run a block's projection-shortcut dgrad after the main branch's (see the block backward):
    a stride-2 shortcut whose input map is large enough for the parity-class dgrad, next to an
    unstrided first main conv (a Bottleneck's 1x1: its plain dgrad loses nothing, while a
    BasicBlock's strided 3x3 needs the operands for its own parity-class dgrad)."""
    from ..ops import kernels as K
    if not _SHORT_LAST:
        return False
    x = short_saved[0]
    if not x.is_cuda or tuple(sc.stride) != (2, 2) or tuple(conv1.stride) != (1, 1):
        return False
    B, H, W, _ = x.shape
    return B * H * W >= K._S2_PARITY_MIN_ROWS


def _out_hw_c(c_in_shape, conv):
    """(OH, OW, Cout) of a 3x3 / s1 / p1 conv on a c_in_shape input (shape-preserving)."""
    return (c_in_shape[1], c_in_shape[2], shadow_of(conv.weight).shape[0])


def _fold_unit(x, plan):
    """Index of the BasicBlock's first unit when its BN + ReLU can run inside the second conv's
    halo patch staging (training, GPU, 3x3/s1 halo-eligible second conv), else None."""
    if not (_BN_FOLD and x.is_cuda):
        return None
    return _fold_unit_shape(tuple(x.shape), plan)


def _fold_unit_shape(xshape, plan):
    from ..ops import kernels as K
    if not _BN_FOLD:
        return None
    mains = [i for i, u in enumerate(plan) if u[3] != "short"]
    if len(mains) != 2:
        return None
    i1, i2 = mains
    conv1, _, relu1, _ = plan[i1]
    conv2 = plan[i2][0]
    if getattr(conv1, "bias", None) is not None or getattr(conv2, "bias", None) is not None:
        return None          # the BN-folding halo conv has no bias epilogue
    if not relu1 or conv2.kernel_size != (3, 3) or tuple(conv2.stride) != (1, 1) or tuple(conv2.padding) != (1, 1):
        return None
    B, H, W, _ = xshape
    kh, kw = conv1.kernel_size
    OH, OW = K.out_hw(H, W, kh, kw, conv1.stride[0], conv1.stride[1], conv1.padding[0], conv1.padding[1])
    shape1 = (B, OH, OW, shadow_of(conv1.weight).shape[0])
    if K.unrolled22(H, W, kh, kw, conv1.stride, conv1.padding) and not _FOLD_UNROLLED:
        return None
    return i1 if K.bnin_ok(shape1, shadow_of(conv2.weight).shape[0], 3, 3, (1, 1), (1, 1)) else None


# the folded conv1 may itself run unrolled (2x2 maps: its folded statistics rows feed the one-shot
# BN-in conv2 like any rows); False: layer3's blocks keep their separate bn1 apply (tests)
_FOLD_UNROLLED = True


def block_params(block) -> List[torch.nn.Parameter]:
    ps = []
    for conv, bn, _, _ in block._kml_plan:
        ps += [conv.weight, bn.weight, bn.bias]
    return ps
