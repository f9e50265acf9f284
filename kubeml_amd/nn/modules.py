"""MI355X-native layers (NHWC bf16 activations, HIP kernels, flat fp32 parameters).

Activation convention: 4-d activations are NHWC.  On an MI355X they are bf16 with
the channel dimension padded to a multiple of 8 (16-byte vectors); on the CPU the
same modules run in fp32 through the stock PyTorch reference ops so the whole
framework (SDK, K-AVG, elastic resize, CLI) is testable without a GPU.

Parameters keep torch's shapes and ``state_dict`` names (``weight`` ``[Cout, Cin,
KH, KW]``, ``bias``, BN ``running_mean`` …) but are views into storage laid out for
the kernels (see :mod:`kubeml_amd.nn.flat`).  Gradients are accumulated by the HIP
kernels directly into ``p.grad`` storage (``+=``), matching torch's semantics.
"""
from __future__ import annotations

import math
from typing import Optional
import os

import torch
import torch.nn as tnn
import torch.nn.functional as F
from torch.autograd import Function

from .flat import grad_out, grad_out_pair, grad_storage_of, master_of, shadow_of


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


def _round8(c):
    return -(-c // 8) * 8


def _on_gpu(x):
    return x.is_cuda


# Large linears (BERT: M = batch x seq tokens) run their three GEMMs on the hand-written
# 256/128-tile LDS-DMA MFMA kernel of csrc/kernels/gemm.hip (ops/gemm.py): bias and erf-GELU
# in the forward epilogue, the weight gradient accumulated in fp32 straight into the flat
# gradient storage (split-K with agent atomics).  Small-M layers and fused-ReLU heads stay on
# the implicit-GEMM conv kernels.


def _linear_route(M, ip, op, act):
    """'gemm' (gemm.hip) or 'conv' (implicit-GEMM kernels)."""
    big = M >= 2048 and ip >= 256 and op >= 256 and act != 1
    return "gemm" if big else "conv"


class _PadChannelsFn(Function):
    """Zero-pad the last dim to ``cp`` (kernel), differentiable (backward slices)."""

    @staticmethod
    def forward(ctx, x, cp):
        from ..ops import kernels as K
        ctx.c = x.shape[-1]
        return K.pad_channels(x.contiguous(), cp)

    @staticmethod
    def backward(ctx, dy):
        return dy[..., :ctx.c].contiguous(), None


def pad_channels(x, cp):
    return _PadChannelsFn.apply(x, cp) if x.requires_grad else _pad_nograd(x, cp)


def _pad_nograd(x, cp):
    from ..ops import kernels as K
    return K.pad_channels(x.contiguous(), cp)


# ======================================================================================
# Conv2d
# ======================================================================================

class _ConvFn(Function):
    @staticmethod
    def forward(ctx, x, weight, bias, mod):
        from ..ops import kernels as K
        w = shadow_of(weight)
        y = K.conv_fwd(x, w, mod.kernel_size[0], mod.kernel_size[1], mod.stride, mod.padding,
                       bias=None if bias is None else master_of(bias))
        ctx.mod = mod
        ctx.x = x
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        from ..ops import kernels as K
        mod = ctx.mod
        dy = dy.contiguous()
        dw, acc = grad_out(mod.weight)
        K.conv_wgrad(ctx.x, dy, dw, mod.kernel_size[0], mod.kernel_size[1], mod.stride, mod.padding, accumulate=acc)
        if ctx.has_bias:
            K.colsum_(dy.view(-1, dy.shape[-1]), grad_storage_of(mod.bias))
        dx = None
        if ctx.needs_input_grad[0]:
            dx = K.conv_dgrad(dy, shadow_of(mod.weight), ctx.x.shape, mod.kernel_size[0],
                              mod.kernel_size[1], mod.stride, mod.padding)
        ctx.x = None
        return dx, None, None, None


class Conv2d(tnn.Module):
    """NHWC convolution on MFMA implicit-GEMM kernels (groups=1, dilation=1)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, bias=True):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.kernel_size = _pair(kernel_size)
        self.stride = _pair(stride)
        self.padding = _pair(padding)
        self.cin_pad = _round8(in_channels)
        # output channels padded to 8 as well (pad filters/bias stay zero, so the extra
        # output channels are exact zeros that the next conv's padded input expects)
        self.cout_pad = _round8(out_channels)
        kh, kw = self.kernel_size
        self.weight = tnn.Parameter(torch.empty(out_channels, in_channels, kh, kw))
        self.bias = tnn.Parameter(torch.empty(out_channels)) if bias else None
        cin, cp, cout = in_channels, self.cin_pad, out_channels
        self.weight._kml_storage_shape = (self.cout_pad, kh, kw, cp)
        self.weight._kml_view = lambda st: st[:cout, :, :, :cin].permute(0, 3, 1, 2)
        if self.bias is not None:
            self.bias._kml_storage_shape = (self.cout_pad,)
            self.bias._kml_view = lambda st: st[:cout]
        self.reset_parameters()

    def reset_parameters(self):
        tnn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            fan_in = self.in_channels * self.kernel_size[0] * self.kernel_size[1]
            b = 1 / math.sqrt(fan_in)
            tnn.init.uniform_(self.bias, -b, b)

    def extra_repr(self):
        return (f"{self.in_channels}, {self.out_channels}, kernel_size={self.kernel_size}, "
                f"stride={self.stride}, padding={self.padding}, bias={self.bias is not None}, layout=NHWC")

    def forward(self, x):
        if not _on_gpu(x):
            y = F.conv2d(x.permute(0, 3, 1, 2), self.weight, self.bias, self.stride, self.padding)
            return y.permute(0, 2, 3, 1)
        if x.shape[-1] != self.cin_pad:
            x = pad_channels(x, self.cin_pad)
        return _ConvFn.apply(x.contiguous(), self.weight, self.bias, self)


# ======================================================================================
# Linear (a 1x1 convolution over a 1x1 image on the same MFMA kernels)
# ======================================================================================

class _LinearFn(Function):
    """act: 0 none, 1 ReLU (implicit-GEMM path), 2 erf-GELU (gemm.hip epilogue; the
    pre-activation is kept for backward)."""

    @staticmethod
    def forward(ctx, x2, weight, bias, mod, act, keep_pad=False):
        from ..ops import kernels as K
        op, ip = mod.out_pad, mod.in_pad
        B = x2.shape[0]
        route = _linear_route(B, ip, op, act)
        ctx.route = route
        object.__setattr__(mod, "_kml_route", route)
        pre = None
        if route == "gemm":
            from ..ops import gemm as G
            w2 = shadow_of(weight).view(op, ip)
            pre = torch.empty((B, op), dtype=torch.bfloat16, device=x2.device) if act == 2 else None
            y = G.linear_fwd(x2, w2, None if bias is None else master_of(bias), act=1 if act == 2 else 0, pre=pre,
                             bias16=None if bias is None else shadow_of(bias))
        else:
            if act == 2:
                raise ValueError("fused GELU needs the large-linear GEMM path")
            w = shadow_of(weight).view(op, 1, 1, ip)
            bias_st = None if bias is None else master_of(bias)
            y = K.conv_fwd(x2.view(B, 1, 1, ip), w, 1, 1, (1, 1), (0, 0), bias=bias_st, relu=act == 1).view(B, op)
        ctx.mod, ctx.x, ctx.has_bias, ctx.act = mod, x2, bias is not None, act
        ctx.y = y if act == 1 else None
        ctx.pre = pre
        # GELU hand-off (models/bert.py): a Linear declared as this one's sole consumer runs
        # the GELU backward in its dgrad epilogue; it finds the pre-activation here
        if pre is not None:
            object.__setattr__(mod, "_kml_gelu_pre", (y.data_ptr(), pre))
        ctx.gelu = None
        prod = getattr(mod, "_kml_gelu_producer", None)
        if prod is not None and route == "gemm":
            hand = getattr(prod, "_kml_gelu_pre", None)
            if hand is not None and hand[0] == x2.data_ptr():
                ctx.gelu = (prod, hand[1])
                object.__setattr__(prod, "_kml_gelu_pre", None)
        ctx.keep_pad = keep_pad
        if op != mod.out_features and not keep_pad:
            y = y[:, :mod.out_features].contiguous()
        return y

    @staticmethod
    def backward(ctx, dy):
        from ..ops import kernels as K
        mod = ctx.mod
        op, ip = mod.out_pad, mod.in_pad
        B = dy.shape[0]
        dy = dy.contiguous()
        if dy.dtype != torch.bfloat16:
            dy = dy.to(torch.bfloat16)
        if op != mod.out_features and dy.shape[1] != op:
            dy = K.pad_channels(dy, op)
        bias_done = False
        if ctx.act == 1:
            dy = K.relu_bwd(dy, ctx.y)
        elif ctx.act == 2:
            if getattr(mod, "_kml_gelu_done", False):
                # the consumer's dgrad already applied the GELU backward and summed the bias
                object.__setattr__(mod, "_kml_gelu_done", False)
            else:
                from ..ops import transformer as T
                # the bias gradient comes out of the GELU backward pass (no column-sum pass)
                dy = T.gelu_bwd(dy, ctx.pre, dbias=grad_storage_of(mod.bias) if ctx.has_bias else None)
            bias_done = ctx.has_bias
        dy4 = dy.view(B, 1, 1, op)
        x4 = ctx.x.view(B, 1, 1, ip)
        if ctx.route == "conv":          # implicit-GEMM wgrad: stores or adds, deterministic
            dwst, wacc = grad_out(mod.weight)
        else:
            from ..ops import gemm as G
            if G.wgrad_can_store(op, ip, B):   # slab split-K / one pass: stores the first write
                dwst, wacc = grad_out(mod.weight)
            else:                              # fp32-atomic split-K: adds only
                dwst, wacc = grad_storage_of(mod.weight), True
        dw4 = dwst.view(op, 1, 1, ip)
        # implicit-GEMM route: the bias gradient is one more column of the wgrad GEMM (a ones
        # column in its input operand) — no column-sum pass
        dbias, bacc = None, True
        if ctx.route == "conv" and ctx.has_bias and not bias_done and not getattr(mod, "_kml_bias_done", False):
            dbias, bacc = grad_out(mod.bias)
            bias_done = True
        dx = None
        # residual gradient handed over by a LayerNorm that shares this Linear's input
        # (nn/transformer.py): summed into dx here instead of by an autograd add
        stash = getattr(mod, "_kml_res_grad", None)
        addend = None
        if stash is not None:
            object.__setattr__(mod, "_kml_res_grad", None)
            if stash[0] != ctx.x.data_ptr():
                raise RuntimeError("residual-gradient hand-off: the LayerNorm residual is not this Linear's input")
            addend = stash[1]
        if ctx.route == "gemm":
            from ..ops import gemm as G
            w2 = shadow_of(mod.weight).view(op, ip)
            if ctx.needs_input_grad[0]:
                dx = None
                if ctx.gelu is not None and addend is None and _GELU_FUSE:
                    prod, pre = ctx.gelu
                    dx = G.linear_dgrad_gelu(dy, w2, pre,
                                             dbias=grad_storage_of(prod.bias) if prod.bias is not None else None)
                    if dx is not None:
                        object.__setattr__(prod, "_kml_gelu_done", True)
                if dx is None:
                    dx = G.linear_dgrad(dy, w2, addend=addend)
                addend = None
            G.linear_wgrad_(dw4.view(op, ip), dy, ctx.x, accumulate=wacc)
        elif ctx.needs_input_grad[0]:
            # dgrad + wgrad as one grouped launch; when this Linear reads a residual block's output
            # directly (a classifier on 1x1 maps: ResNet on 32x32 input), the dgrad epilogue also
            # emits that block's output-BN partial rows and applies its ReLU mask, so the block's
            # BN backward skips its reduction pass (the nn/fused.py block-to-block hand-off)
            w = shadow_of(mod.weight).view(op, 1, 1, ip)
            blk = getattr(mod, "_kml_bnf_block", None)
            saved = getattr(blk, "_kml_last_saved", None) if blk is not None else None
            bnf = None
            if (saved is not None and saved[2] is not None and addend is None and ctx.x.is_cuda and
                    tuple(saved[1].shape) == (B, 1, 1, ip) and saved[2].data_ptr() == ctx.x.data_ptr()):
                bnf = (saved[2], saved[1], saved[3], saved[4])
            r = K.conv_bwd(dy4, w, x4, dw4, 1, 1, (1, 1), (0, 0), accumulate=wacc, dbias=dbias,
                           bias_accumulate=bacc, bnf=bnf, bnf_mask=bnf is not None)
            if bnf is not None:
                r, part = r
                object.__setattr__(blk, "_kml_in_partial", (r.data_ptr(), part))
            dx = r.view(B, ip)
        else:
            K.conv_wgrad(x4, dy4, dw4, 1, 1, (1, 1), (0, 0), accumulate=wacc, dbias=dbias, bias_accumulate=bacc)
        if ctx.has_bias and not bias_done:
            if getattr(mod, "_kml_bias_done", False):
                object.__setattr__(mod, "_kml_bias_done", False)   # summed by the consumer LayerNorm
            else:
                K.colsum_(dy, grad_storage_of(mod.bias))
        if addend is not None and dx is not None:
            dx = K.add_bf16(dx, addend)
        ctx.x = ctx.y = ctx.pre = ctx.gelu = None
        return dx, None, None, None, None, None


# FFN1 -> FFN2: FFN2's dgrad epilogue applies FFN1's GELU backward (ops.gemm.linear_dgrad_gelu)
_GELU_FUSE = True


class Linear(tnn.Module):
    def __init__(self, in_features, out_features, bias=True, fused_relu=False):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.in_pad = _round8(in_features)
        self.out_pad = _round8(out_features)
        self.fused_relu = fused_relu
        self.weight = tnn.Parameter(torch.empty(out_features, in_features))
        self.bias = tnn.Parameter(torch.empty(out_features)) if bias else None
        # storage padded to 16-byte rows/columns for the MFMA kernels (pad entries stay 0)
        inf, outf = in_features, out_features
        self.weight._kml_storage_shape = (self.out_pad, self.in_pad)
        self.weight._kml_view = lambda st: st[:outf, :inf]
        if self.bias is not None:
            self.bias._kml_storage_shape = (self.out_pad,)
            self.bias._kml_view = lambda st: st[:outf]
        self.reset_parameters()

    def reset_parameters(self):
        tnn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            b = 1 / math.sqrt(self.in_features)
            tnn.init.uniform_(self.bias, -b, b)

    def extra_repr(self):
        return f"in_features={self.in_features}, out_features={self.out_features}, bias={self.bias is not None}"

    def forward(self, x, act: Optional[str] = None, keep_pad: bool = False):
        """act: None (module default: fused ReLU if constructed so), "gelu" (erf-GELU fused
        into the GEMM epilogue on the GPU).  keep_pad: on the GPU return the [N, out_pad]
        output whose columns past out_features are zero (no slice copy; a consumer that
        knows the real width — ``cross_entropy(classes=...)`` — uses it in place)."""
        a = 2 if act == "gelu" else (1 if self.fused_relu else 0)
        if not _on_gpu(x):
            y = F.linear(x, self.weight, self.bias)
            return F.relu(y) if a == 1 else (F.gelu(y) if a == 2 else y)
        if x.dim() != 2:
            x = x.reshape(x.shape[0], -1)
        if x.dtype != torch.bfloat16:
            x = x.to(torch.bfloat16)
        if x.shape[1] != self.in_pad:
            x = pad_channels(x, self.in_pad)
        if a == 2 and _linear_route(x.shape[0], self.in_pad, self.out_pad, 2) != "gemm":
            from .transformer import GELU
            return GELU()(_LinearFn.apply(x.contiguous(), self.weight, self.bias, self, 0))
        y = _LinearFn.apply(x.contiguous(), self.weight, self.bias, self, a, keep_pad)
        if a == 0:
            y._kml_linear = self   # raw linear output: a consuming cross_entropy may sum our bias grad
        return y


# ======================================================================================
# BatchNorm2d (+ fused ReLU / residual)
# ======================================================================================

class _BNFn(Function):
    @staticmethod
    def forward(ctx, x, weight, bias, mod, relu, res):
        from ..ops import kernels as K
        C = x.shape[-1]
        stats, G = K.bn_stats_part(x.view(-1, C))
        mean = torch.empty(C, dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        y = K.bn_apply(x, stats, master_of(weight), master_of(bias), res=res, save_mean=mean, save_rstd=rstd,
                       stats_rows=G,
                       run_mean=mod.running_mean if mod.track_running_stats else None,
                       run_var=mod.running_var if mod.track_running_stats else None,
                       eps=mod.eps, momentum=mod.momentum if mod.momentum is not None else 0.1, relu=relu)
        ctx.mod, ctx.x, ctx.y, ctx.mean, ctx.rstd, ctx.relu, ctx.has_res = mod, x, y, mean, rstd, relu, res is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        from ..ops import kernels as K
        mod = ctx.mod
        dy = dy.contiguous()
        dres = torch.empty_like(dy) if ctx.has_res else None
        dg, db, acc = grad_out_pair(mod.weight, mod.bias)
        dx = K.bn_bwd(dy, ctx.y if ctx.relu else None, ctx.x, ctx.mean, ctx.rstd, master_of(mod.weight),
                      dg, db, dres=dres, accumulate=acc)
        ctx.x = ctx.y = None
        return dx, None, None, None, None, dres


class BatchNorm2d(tnn.BatchNorm2d):
    """torch.nn.BatchNorm2d semantics and state_dict, NHWC input, HIP kernels on GPU."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, track_running_stats=True):
        super().__init__(num_features, eps, momentum, affine, track_running_stats)
        if not affine:
            raise NotImplementedError("affine=False is not supported by the fused kernels")

    def forward(self, x, relu=False, residual=None):
        if not _on_gpu(x):
            y = F.batch_norm(x.permute(0, 3, 1, 2), self.running_mean, self.running_var, self.weight, self.bias,
                             self.training or not self.track_running_stats, self.momentum or 0.1, self.eps)
            y = y.permute(0, 2, 3, 1)
            if self.training and self.track_running_stats:
                self.num_batches_tracked.add_(1)
            if residual is not None:
                y = y + residual
            return F.relu(y) if relu else y
        x = x.contiguous()
        if self.training or not self.track_running_stats:
            if self.track_running_stats:
                from ..ops import kernels as K
                K.add_i64_(self.num_batches_tracked)
            return _BNFn.apply(x, self.weight, self.bias, self, relu, residual)
        from ..ops import kernels as K
        return K.bn_apply(x, None, master_of(self.weight), master_of(self.bias), res=residual,
                          run_mean=self.running_mean, run_var=self.running_var, eps=self.eps, relu=relu,
                          training=False)


# ======================================================================================
# activations / pooling / shape
# ======================================================================================

class _ReLUFn(Function):
    @staticmethod
    def forward(ctx, x):
        from ..ops import kernels as K
        y = K.relu_fwd(x)
        ctx.y = y
        return y

    @staticmethod
    def backward(ctx, dy):
        from ..ops import kernels as K
        dx = K.relu_bwd(dy.contiguous(), ctx.y)
        ctx.y = None
        return dx


class ReLU(tnn.Module):
    def __init__(self, inplace=False):
        super().__init__()

    def forward(self, x):
        if not _on_gpu(x) or x.numel() % 8 or x.dtype != torch.bfloat16:
            return F.relu(x)
        return _ReLUFn.apply(x.contiguous())


class _MaxPoolFn(Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        from ..ops import kernels as K
        y, idx = K.maxpool_fwd(x, k, s, p)
        ctx.idx, ctx.shape, ctx.kp = idx, x.shape, (k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        from ..ops import kernels as K
        k, s, p = ctx.kp
        dx = K.maxpool_bwd(dy.contiguous(), ctx.idx, ctx.shape, k, s, p)
        ctx.idx = None
        return dx, None, None, None


class MaxPool2d(tnn.Module):
    def __init__(self, kernel_size, stride=None, padding=0):
        super().__init__()
        self.kernel_size = kernel_size
        self.stride = stride if stride is not None else kernel_size
        self.padding = padding

    def extra_repr(self):
        return f"kernel_size={self.kernel_size}, stride={self.stride}, padding={self.padding}"

    def forward(self, x):
        if not _on_gpu(x):
            return F.max_pool2d(x.permute(0, 3, 1, 2), self.kernel_size, self.stride, self.padding).permute(0, 2, 3, 1)
        return _MaxPoolFn.apply(x.contiguous(), self.kernel_size, self.stride, self.padding)


class _GAvgFn(Function):
    @staticmethod
    def forward(ctx, x):
        from ..ops import kernels as K
        ctx.shape = x.shape
        return K.gavgpool_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        from ..ops import kernels as K
        return K.gavgpool_bwd(dy.contiguous(), ctx.shape)


class AdaptiveAvgPool2d(tnn.Module):
    """Only output_size=1 (global average); returns [B, C]."""

    def __init__(self, output_size=(1, 1)):
        super().__init__()
        if _pair(output_size) != (1, 1):
            raise NotImplementedError("only global average pooling is supported")

    def forward(self, x):
        B, H, W, C = x.shape
        if not _on_gpu(x):
            return x.mean((1, 2))
        if H * W == 1:
            return x.reshape(B, C)  # 1x1 spatial (ResNet on 32x32 input): pooling is the identity
        return _GAvgFn.apply(x.contiguous())


class Flatten(tnn.Module):
    def forward(self, x):
        if x.dim() == 4:  # NHWC -> match torch's NCHW flatten order
            if _on_gpu(x) and x.shape[1] * x.shape[2] == 1:
                return x.reshape(x.shape[0], -1)
            return x.permute(0, 3, 1, 2).reshape(x.shape[0], -1)
        return x.reshape(x.shape[0], -1)


def to_nhwc(x, cin_pad=None):
    """User NCHW input -> the layers' activation layout for its device."""
    if x.dim() != 4:
        return x
    if x.is_cuda:
        from ..ops import kernels as K
        if x.dtype == torch.bfloat16 and x.shape[-1] % 8 == 0 and x.is_contiguous():
            return x  # already NHWC bf16
        return K.nchw_to_nhwc_bf16(x, cin_pad)
    y = x.permute(0, 2, 3, 1)
    return y if y.is_floating_point() else y.float()


# ======================================================================================
# loss
# ======================================================================================

class _CEFn(Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index, classes=None, lin=None):
        from ..ops import kernels as K
        out3, ws, lab = K.ce_fwd(logits, labels, ignore_index, classes=classes)
        ctx.save = (logits, lab, ws, out3, ignore_index, classes)
        ctx.out3 = out3
        ctx.lin = lin
        return out3[0]

    @staticmethod
    def backward(ctx, g):
        from ..ops import kernels as K
        logits, lab, ws, out3, ig, classes = ctx.save
        # the logits came straight out of a Linear: its bias gradient (the column sums of
        # dlogits) is added by the CE backward pass itself, and the Linear skips its own —
        # unless the Linear runs on the implicit-GEMM route, whose wgrad GEMM produces the bias
        # gradient as one extra column for free
        lin, dbias, acc = ctx.lin, None, True
        if (lin is not None and getattr(lin, "bias", None) is not None and _CE_BIAS_FUSE
                and getattr(lin, "_kml_route", None) != "conv"
                and lin.out_pad == logits.shape[1] and K.ce_bias_fusable(logits)):
            dbias, acc = grad_out(lin.bias)
            object.__setattr__(lin, "_kml_bias_done", True)
        d = K.ce_bwd(logits, lab, ws, out3, grad_out=g.reshape(1).float().contiguous(), ignore_index=ig,
                     classes=classes, dbias=dbias, accumulate=acc)
        ctx.save = ctx.lin = None
        return d, None, None, None, None


_CE_BIAS_FUSE = True    # the head's bias gradient comes out of the cross-entropy backward


def cross_entropy(logits, labels, ignore_index=-100, return_correct=False, classes=None):
    """Mean softmax cross-entropy (fused HIP kernel on GPU).  With return_correct the
    device-side argmax==label count of the same pass is returned as well.  ``classes``:
    the real class count when ``logits`` rows are padded past it (a ``keep_pad`` Linear
    output; the pad columns are ignored and get a zero gradient)."""
    if not logits.is_cuda:
        if classes is not None:
            logits = logits[:, :classes]
        loss = F.cross_entropy(logits.float(), labels, ignore_index=ignore_index)
        if return_correct:
            valid = labels != ignore_index
            return loss, (logits.argmax(1) == labels)[valid].sum().float()
        return loss
    if return_correct:
        from ..ops import kernels as K
        if torch.is_grad_enabled() and logits.requires_grad:
            loss = _CEFn.apply(logits.contiguous(), labels, ignore_index, classes, getattr(logits, "_kml_linear", None))
            return loss, loss.grad_fn.out3[1]  # grad_fn is the Function ctx; same fused pass
        out3, _, _ = K.ce_fwd(logits.contiguous(), labels, ignore_index, classes=classes)
        return out3[0], out3[1]
    return _CEFn.apply(logits.contiguous(), labels, ignore_index, classes, getattr(logits, "_kml_linear", None))


_ONES: dict = {}


def backward_loss(loss):
    """``loss.backward()`` without autograd's seed-gradient fill launch: the seed is a
    cached device constant, so a captured training step has one kernel less."""
    if not loss.is_cuda or loss.numel() != 1:
        loss.backward()
        return
    key = (loss.device, loss.dtype, tuple(loss.shape))
    one = _ONES.get(key)
    if one is None:
        one = _ONES[key] = torch.ones_like(loss)
    torch.autograd.backward(loss, one)


class CrossEntropyLoss(tnn.Module):
    def __init__(self, ignore_index=-100):
        super().__init__()
        self.ignore_index = ignore_index

    def forward(self, logits, labels):
        return cross_entropy(logits, labels, self.ignore_index)
