"""Transformer layers on the MI355X kernels (token-major ``[T, hidden]`` bf16 on GPU,
fp32 stock-torch path on CPU with identical parameters / ``state_dict`` names).

* :class:`LayerNorm`     — torch.nn.LayerNorm semantics; fused residual add
* :class:`GELU`, :class:`Dropout` — erf GELU; counter-based dropout (mask regenerated
  in backward from a device ``[seed, step]`` pair, so graph replays draw new masks)
* :class:`SelfAttention` — fused QKV projection (one GEMM, ``[T, 3H]``) + flash
  attention kernel + output projection; ``state_dict`` exposes HuggingFace's
  ``query/key/value`` names via state-dict hooks
* :class:`Embeddings`    — word + position + token-type gather and LayerNorm
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as tnn
import torch.nn.functional as F
from torch.autograd import Function

from .flat import grad_storage_of, master_of, shadow_of
from .modules import Linear


def _bf(x):
    return x if x.dtype == torch.bfloat16 else x.to(torch.bfloat16)


# residual gradients summed in the consuming Linear's dgrad epilogue (False: by autograd, a
# separate add; tests compare the two)
_RES_FUSE = True


# ====================================================================================== LayerNorm
class _LNFn(Function):
    @staticmethod
    def forward(ctx, x, weight, bias, mod, res, drop=None, sep_dropout=False):
        from ..ops import transformer as T
        y, xin, mean, rstd = T.ln_fwd(x, master_of(weight), master_of(bias), res=res, eps=mod.eps, drop=drop)
        ctx.save = (xin, mean, rstd)
        ctx.mod = mod
        ctx.has_res = res is not None
        ctx.res_ptr = res.data_ptr() if res is not None else None
        ctx.drop = drop
        ctx.sep_dropout = sep_dropout   # x came through a separate Dropout (not the Linear output)
        return y

    @staticmethod
    def backward(ctx, dy):
        from ..ops import transformer as T
        xin, mean, rstd = ctx.save
        mod = ctx.mod
        # bias gradient of the Linear whose output is this LN's input (``_kml_in_linear``):
        # summed from the input gradient inside the LN backward; that Linear then skips its
        # own column-sum pass (``_kml_bias_done``)
        lin_in = getattr(mod, "_kml_in_linear", None) if _RES_FUSE and not ctx.sep_dropout else None
        dbias = None
        if lin_in is not None and getattr(lin_in, "bias", None) is not None and lin_in.out_pad == xin.shape[-1]:
            dbias = grad_storage_of(lin_in.bias)
            object.__setattr__(lin_in, "_kml_bias_done", True)
        r = T.ln_bwd(_bf(dy).contiguous(), xin, mean, rstd, master_of(mod.weight), grad_storage_of(mod.weight),
                     grad_storage_of(mod.bias), drop=ctx.drop, dbias_in=dbias)
        dx, dxin = r if ctx.drop is not None else (r, r)   # dxin: gradient of the (pre-dropout) input
        ctx.save = ctx.drop = None
        dres = dx if ctx.has_res else None
        lin = getattr(mod, "_kml_res_linear", None)
        if dres is not None and lin is not None and _RES_FUSE:
            # the residual also feeds ``lin`` (whose backward runs next on this path): hand it
            # this gradient so its dgrad GEMM adds it in the epilogue (no separate add kernel)
            object.__setattr__(lin, "_kml_res_grad", (ctx.res_ptr, dres))
            dres = None
        return dxin, None, None, None, dres, None, None


class LayerNorm(tnn.LayerNorm):
    """LayerNorm over the last dim; ``forward(x, residual, dropout)`` normalises
    ``dropout(x) + residual``.  On the GPU in training the dropout runs inside the LayerNorm
    kernels (same counter-hash mask as :class:`Dropout`): no separate dropout pass forward
    or backward (``_LN_DROP_FUSE = False`` keeps it separate)."""

    def forward(self, x, residual=None, dropout=None):
        drop, sep = None, False
        if dropout is not None and dropout.training and dropout.p > 0.0:
            if x.is_cuda and _LN_DROP_FUSE:
                drop = (dropout.rng.tensor(x.device), dropout.salt, dropout.p)
            else:
                x = dropout(x)
                sep = True
        if not x.is_cuda:
            if residual is not None:
                x = x + residual
            return F.layer_norm(x, self.normalized_shape, self.weight, self.bias, self.eps)
        shp = x.shape
        x2 = _bf(x).reshape(-1, shp[-1]).contiguous()
        r2 = None if residual is None else _bf(residual).reshape(-1, shp[-1]).contiguous()
        return _LNFn.apply(x2, self.weight, self.bias, self, r2, drop, sep).view(shp)


_LN_DROP_FUSE = True


class _GELUFn(Function):
    @staticmethod
    def forward(ctx, x):
        from ..ops import transformer as T
        ctx.x = x
        return T.gelu_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        from ..ops import transformer as T
        dx = T.gelu_bwd(_bf(dy).contiguous(), ctx.x)
        ctx.x = None
        return dx


class GELU(tnn.Module):
    def forward(self, x):
        if not x.is_cuda:
            return F.gelu(x)
        return _GELUFn.apply(_bf(x).contiguous())


class RNGState:
    """Device-resident ``[seed, step]`` shared by the dropout layers of one model;
    ``advance()`` (one tiny kernel) runs at the start of every training forward."""

    def __init__(self, seed: int = 0):
        self.seed = seed
        self.t = None

    def tensor(self, device):
        if self.t is None or self.t.device != device:
            self.t = torch.tensor([float(self.seed), 0.0], dtype=torch.float32, device=device)
        return self.t

    def advance(self, device):
        from ..ops import kernels as K
        K.increment_(self.tensor(device)[1:], 1.0)


class _DropFn(Function):
    @staticmethod
    def forward(ctx, x, ctr, salt, p):
        from ..ops import transformer as T
        ctx.args = (ctr, salt, p)
        return T.dropout(x, ctr, salt, p)

    @staticmethod
    def backward(ctx, dy):
        from ..ops import transformer as T
        ctr, salt, p = ctx.args
        return T.dropout(_bf(dy).contiguous(), ctr, salt, p), None, None, None


class Dropout(tnn.Module):
    _salt = 0

    def __init__(self, p: float = 0.1, rng: Optional[RNGState] = None):
        super().__init__()
        self.p = p
        self.rng = rng or RNGState()
        Dropout._salt += 1
        self.salt = Dropout._salt * 7919

    def forward(self, x):
        if not self.training or self.p == 0.0:
            return x
        if not x.is_cuda:
            return F.dropout(x, self.p, True)
        return _DropFn.apply(_bf(x).contiguous(), self.rng.tensor(x.device), self.salt, self.p)


# ====================================================================================== attention
class _AttnFn(Function):
    @staticmethod
    def forward(ctx, qkv, B, H, L, bias, drop=None):
        from ..ops import transformer as T
        D = H * 64
        q, k, v = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
        keep = T.attn_keep_buffer(B, H, L, qkv.device) if drop is not None and drop[2] > 0.0 else None
        out, lse = T.attn_fwd(q, k, v, B, H, L, bias=bias, drop=drop, keep=keep)
        ctx.save = (qkv, out, lse, bias, keep)
        ctx.dims = (B, H, L)
        ctx.drop = drop
        return out

    @staticmethod
    def backward(ctx, dout):
        from ..ops import transformer as T
        qkv, out, lse, bias, keep = ctx.save
        B, H, L = ctx.dims
        D = H * 64
        dqkv = torch.empty_like(qkv)
        T.attn_bwd(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], out, _bf(dout).contiguous(), lse, B, H, L, bias=bias,
                   dq=dqkv[:, :D], dk=dqkv[:, D:2 * D], dv=dqkv[:, 2 * D:], drop=ctx.drop, keep=keep)
        ctx.save = None
        return dqkv, None, None, None, None, None


def attention_reference(qkv, B, H, L, bias=None, keep=None):
    """fp32 torch attention on a fused [B*L, 3*H*64] buffer (CPU path / tests); keep:
    optional [B, H, L, L] dropout multiplier (0 or 1/(1-p)) applied to the probabilities."""
    D = H * 64
    q, k, v = (qkv[:, i * D:(i + 1) * D].reshape(B, L, H, 64).permute(0, 2, 1, 3) for i in range(3))
    s = q @ k.transpose(-1, -2) / math.sqrt(64)
    if bias is not None:
        s = s + bias.view(B, 1, 1, L)
    pr = s.softmax(-1)
    if keep is not None:
        pr = pr * keep
    o = pr @ v
    return o.permute(0, 2, 1, 3).reshape(B * L, D)


def attention_reference_dropout(qkv, B, H, L, bias, p):
    """CPU attention with probability dropout (torch RNG; same semantics as the kernel)."""
    keep = (torch.rand(B, H, L, L) >= p).float() / (1.0 - p)
    return attention_reference(qkv, B, H, L, bias, keep=keep)


class SelfAttention(tnn.Module):
    """BERT self-attention + output projection.  Parameters: one fused ``qkv`` Linear
    ([3H, H]) and ``out`` Linear; ``state_dict`` uses HF names
    (``self.query.weight`` ... ``output.dense.weight``) through hooks."""

    def __init__(self, hidden: int = 768, heads: int = 12, prefix_self: str = "self.", prefix_out: str = "output.dense.",
                 post_ln_eps: Optional[float] = None, prefix_ln: str = "output.LayerNorm.", attn_dropout: float = 0.0,
                 rng: Optional["RNGState"] = None):
        super().__init__()
        # attention-probability dropout (HF attention_probs_dropout_prob), inside the kernel
        self.attn_dropout = float(attn_dropout)
        self.rng = rng or RNGState()
        Dropout._salt += 1
        self.salt = Dropout._salt * 7919
        if hidden != heads * 64:
            raise ValueError("the fused attention kernel needs head_dim 64")
        self.hidden, self.heads = hidden, heads
        self.qkv = Linear(hidden, 3 * hidden)
        self.out = Linear(hidden, hidden)
        self.ln = LayerNorm(hidden, eps=post_ln_eps) if post_ln_eps is not None else None
        self._ps, self._po, self._pl = prefix_self, prefix_out, prefix_ln
        self._register_state_dict_hook(SelfAttention._sd_hook)
        self._register_load_state_dict_pre_hook(SelfAttention._load_hook, with_module=True)

    @staticmethod
    def _sd_hook(mod, sd, prefix, local_metadata):
        H = mod.hidden
        for kind in ("weight", "bias"):
            t = sd.pop(prefix + f"qkv.{kind}")
            for i, n in enumerate(("query", "key", "value")):
                sd[prefix + f"{mod._ps}{n}.{kind}"] = t[i * H:(i + 1) * H]
            sd[prefix + f"{mod._po}{kind}"] = sd.pop(prefix + f"out.{kind}")
            if mod.ln is not None:
                sd[prefix + f"{mod._pl}{kind}"] = sd.pop(prefix + f"ln.{kind}")
        return sd

    @staticmethod
    def _load_hook(mod, sd, prefix, local_metadata, strict, missing, unexpected, errors):
        for kind in ("weight", "bias"):
            names = [prefix + f"{mod._ps}{n}.{kind}" for n in ("query", "key", "value")]
            if all(n in sd for n in names):
                sd[prefix + f"qkv.{kind}"] = torch.cat([sd.pop(n) for n in names], 0)
            on = prefix + f"{mod._po}{kind}"
            if on in sd:
                sd[prefix + f"out.{kind}"] = sd.pop(on)
            ln = prefix + f"{mod._pl}{kind}"
            if mod.ln is not None and ln in sd:
                sd[prefix + f"ln.{kind}"] = sd.pop(ln)

    def forward(self, x, B: int, L: int, bias=None):
        qkv = self.qkv(x)
        if not x.is_cuda:
            if self.training and self.attn_dropout > 0:
                ctx = attention_reference_dropout(qkv, B, self.heads, L, bias, self.attn_dropout)
            else:
                ctx = attention_reference(qkv, B, self.heads, L, bias)
        else:
            drop = None
            if self.training and self.attn_dropout > 0:
                drop = (self.rng.tensor(x.device), self.salt, self.attn_dropout)
            ctx = _AttnFn.apply(qkv.contiguous(), B, self.heads, L, bias, drop)
        return self.out(ctx)


# ====================================================================================== embeddings
class _EmbFn(Function):
    @staticmethod
    def forward(ctx, ids, tt, wword, wpos, wtype, mod, L):
        from ..ops import transformer as T
        out = T.embed_fwd(ids, tt, shadow_of(wword), shadow_of(wpos), shadow_of(wtype), L)
        ctx.save = (ids, tt)
        ctx.mod, ctx.L = mod, L
        return out

    @staticmethod
    def backward(ctx, dsum):
        from ..ops import transformer as T
        ids, tt = ctx.save
        m = ctx.mod
        T.embed_bwd(ids, tt, _bf(dsum).contiguous(), grad_storage_of(m.word_embeddings.weight),
                    grad_storage_of(m.position_embeddings.weight), grad_storage_of(m.token_type_embeddings.weight),
                    ctx.L)
        ctx.save = None
        return (None,) * 7


class Embeddings(tnn.Module):
    def __init__(self, vocab: int = 30522, hidden: int = 768, max_pos: int = 512, type_vocab: int = 2,
                 eps: float = 1e-12, dropout: float = 0.1, rng: Optional[RNGState] = None):
        super().__init__()
        self.word_embeddings = tnn.Embedding(vocab, hidden)
        self.position_embeddings = tnn.Embedding(max_pos, hidden)
        self.token_type_embeddings = tnn.Embedding(type_vocab, hidden)
        self.LayerNorm = LayerNorm(hidden, eps=eps)
        self.dropout = Dropout(dropout, rng)
        # storage rows padded to 8 so the tied decoder Linear can share the word table
        vp = -(-vocab // 8) * 8
        self.word_embeddings.weight._kml_storage_shape = (vp, hidden)
        self.word_embeddings.weight._kml_view = lambda st: st[:vocab, :hidden]

    def forward(self, ids, token_type_ids=None):
        B, L = ids.shape
        if not ids.is_cuda:
            pos = torch.arange(L, device=ids.device)
            tt = token_type_ids if token_type_ids is not None else torch.zeros_like(ids)
            e = self.word_embeddings(ids) + self.position_embeddings(pos)[None] + self.token_type_embeddings(tt)
            e = e.reshape(B * L, -1)
        else:
            tt = token_type_ids.reshape(-1).contiguous() if token_type_ids is not None else None
            e = _EmbFn.apply(ids.reshape(-1).contiguous(), tt, self.word_embeddings.weight,
                             self.position_embeddings.weight, self.token_type_embeddings.weight, self, L)
        return self.dropout(self.LayerNorm(e))


# ====================================================================================== row gather
class _GatherFn(Function):
    @staticmethod
    def forward(ctx, x, idx):
        from ..ops import transformer as T
        ctx.save = (idx, x.shape)
        return T.gather_rows(x, idx)

    @staticmethod
    def backward(ctx, dy):
        from ..ops import kernels as K
        from ..ops import transformer as T
        idx, shp = ctx.save
        dx = torch.empty(shp, dtype=torch.bfloat16, device=dy.device)
        K.memset_(dx)
        T.scatter_rows(_bf(dy).contiguous(), idx, dx)
        return dx, None


def gather_rows(x, idx):
    """rows ``x[idx]`` (idx unique) with a scatter backward."""
    if not x.is_cuda:
        return x[idx]
    return _GatherFn.apply(x.contiguous(), idx)
