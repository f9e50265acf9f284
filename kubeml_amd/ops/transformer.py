"""Launchers for the transformer kernels (csrc/kernels/attention.hip, transformer.hip).

All take/return token-major bf16 tensors ``[T, N]`` (T = batch x seq), fp32 statistics
and fp32 gradient accumulators; every launch goes on the current HIP stream and is
hipGraph-capturable (no host sync, no memset nodes).
"""
from __future__ import annotations

import math

import os

import torch

from .._native import HIP
from .kernels import BF16, F32, _COUNTERS, _chk, _p, _s

I64 = torch.int64


def _chk_view(t, name):
    """bf16 GPU row-major 2-d view (column slices of a wider buffer allowed)."""
    if t.dtype != BF16:
        raise TypeError(f"{name}: expected bfloat16, got {t.dtype}")
    if not t.is_cuda:
        raise ValueError(f"{name}: must be a GPU tensor")
    if t.dim() != 2 or t.stride(1) != 1 or t.stride(0) % 8 or t.data_ptr() % 16:
        raise ValueError(f"{name}: expected a 16-byte aligned row-major 2-d view, got stride {t.stride()}")


def _drop_args(drop):
    """drop = (ctr [seed, step] device tensor, salt, p) or None."""
    if drop is None or drop[2] <= 0.0:
        return 0, 0, 0.0
    ctr, salt, p = drop
    _chk(ctr, F32, "ctr")
    if not 0.0 <= p < 1.0:
        raise ValueError("dropout p must be in [0, 1)")
    return ctr.data_ptr(), int(salt) & 0x7FFFFFFF, float(p)


def attn_keep_buffer(B, H, L, device):
    """Buffer for the attention-dropout keep bits the forward writes and the backward reads
    (attention.hip ``Drop``): one u64 word per (b*h, key tile, query), queries padded to
    whole 64-row tiles — B*H*L^2/8 bytes, 12.6 MB per BERT-base layer at L = 512."""
    nkb = (L + 63) // 64
    return torch.empty(B * H * nkb * nkb * 64 * 8, dtype=torch.uint8, device=device)


def _keep_arg(keep, B, H, L, drop):
    if keep is None or drop is None or drop[2] <= 0.0:
        return 0
    nkb = (L + 63) // 64
    if keep.dtype != torch.uint8 or not keep.is_cuda or keep.numel() < B * H * nkb * nkb * 512:
        raise ValueError("keep must be a GPU uint8 buffer from attn_keep_buffer(B, H, L)")
    return keep.data_ptr()


def attn_fwd(q, k, v, B, H, L, bias=None, out=None, scale=None, drop=None, keep=None):
    """q/k/v: [B*L, ld] bf16 views with head h at columns 64h..64h+63 (may be column
    slices of one fused QKV buffer).  drop: (ctr, salt, p) attention-probability dropout;
    keep: optional :func:`attn_keep_buffer` that receives the dropout keep bits, so
    :func:`attn_bwd` reads them instead of re-hashing.  Returns (out [B*L, H*64], lse [B*H, L])."""
    for n, t in (("q", q), ("k", k), ("v", v)):
        _chk_view(t, n)
        if t.shape[0] != B * L or t.shape[1] < H * 64:
            raise ValueError(f"{n}: expected a row-major [B*L, >= {H * 64}] view, got {tuple(t.shape)}")
    if bias is not None:
        _chk(bias, F32, "bias")
        if bias.numel() != B * L:
            raise ValueError("bias must be [B, L]")
    if out is None:
        out = torch.empty((B * L, H * 64), dtype=BF16, device=q.device)
    lse = torch.empty((B * H, L), dtype=F32, device=q.device)
    scale = 1.0 / math.sqrt(64) if scale is None else scale
    c, salt, pd = _drop_args(drop)
    HIP.call("kml_attn_fwd", "p p p p p p i i i i i i i f p i f p s", _p(q), _p(k), _p(v), _p(out), _p(lse),
             _p(bias), q.stride(0), k.stride(0), v.stride(0), out.stride(0), B, H, L, float(scale), c, salt, pd,
             _keep_arg(keep, B, H, L, drop), _s())
    return out, lse


def attn_bwd(q, k, v, o, dout, lse, B, H, L, bias=None, dq=None, dk=None, dv=None, scale=None, drop=None,
             keep=None):
    """Gradients of attention; dq/dk/dv may be column views of one [B*L, 3*H*64] buffer.
    keep: the keep-bit buffer the forward filled (same drop), or None to re-hash the mask."""
    dev = q.device
    if dq is None:
        dq = torch.empty((B * L, H * 64), dtype=BF16, device=dev)
    if dk is None:
        dk = torch.empty((B * L, H * 64), dtype=BF16, device=dev)
    if dv is None:
        dv = torch.empty((B * L, H * 64), dtype=BF16, device=dev)
    for n, t in (("q", q), ("k", k), ("v", v), ("o", o), ("dout", dout), ("dq", dq), ("dk", dk), ("dv", dv)):
        _chk_view(t, n)
        if t.shape[0] != B * L or t.shape[1] < H * 64:
            raise ValueError(f"{n}: expected [B*L, >= {H * 64}], got {tuple(t.shape)}")
    if lse.shape != (B * H, L) or lse.dtype != F32:
        raise ValueError("lse must be fp32 [B*H, L] from attn_fwd")
    dsum = torch.empty((B * H, L), dtype=F32, device=dev)
    scale = 1.0 / math.sqrt(64) if scale is None else scale
    c, salt, pd = _drop_args(drop)
    HIP.call("kml_attn_bwd", "p p p p p p p p p p p i i i i i i i i i i i f p i f p s",
             _p(q), _p(k), _p(v), _p(o), _p(dout), _p(lse), _p(dsum), _p(bias), _p(dq), _p(dk), _p(dv),
             q.stride(0), k.stride(0), v.stride(0), o.stride(0), dout.stride(0), dq.stride(0), dk.stride(0),
             dv.stride(0), B, H, L, float(scale), c, salt, pd, _keep_arg(keep, B, H, L, drop), _s())
    return dq, dk, dv


def ln_fwd(x, gamma, beta, res=None, eps=1e-12, keep_sum=True, drop=None):
    """LayerNorm over the last dim of a [T, N] bf16 tensor (optionally of x + res).
    Returns (y, ln_input, mean, rstd) — ln_input is x + res (or x).  drop = (ctr, salt, p):
    x goes through :func:`dropout` (same mask) as it is loaded — LN(dropout(x) + res) in one
    pass; ln_input is then dropout(x) + res."""
    _chk(x, BF16, "x")
    N = x.shape[-1]
    M = x.numel() // N
    y = torch.empty_like(x)
    s = torch.empty_like(x) if ((res is not None or drop is not None) and keep_sum) else None
    mean = torch.empty(M, dtype=F32, device=x.device)
    rstd = torch.empty(M, dtype=F32, device=x.device)
    ctr, salt, p = drop if drop is not None else (None, 0, 0.0)
    HIP.call("kml_ln_fwd", "p p p p p p p p l i f p i f s", _p(x), _p(res), _p(gamma), _p(beta), _p(y), _p(s),
             _p(mean), _p(rstd), M, N, float(eps), _p(ctr), int(salt) & 0x7FFFFFFF, float(p), _s())
    return y, (s if s is not None else x), mean, rstd


def ln_bwd(dy, xin, mean, rstd, gamma, dgamma, dbeta, dx_add=None, drop=None, dbias_in=None):
    """dx (+ dx_add) ; dgamma/dbeta += (deterministic two-level reduce).  drop = (ctr, salt,
    p) of a forward :func:`ln_fwd` dropout: returns (dx, dropout(dx)) — the gradients of the
    residual input and of the pre-dropout input — from one pass.  dbias_in (fp32 [N]) +=
    column sums of the input gradient: the bias gradient of the Linear feeding the LN."""
    _chk(dy, BF16, "dy")
    N = dy.shape[-1]
    M = dy.numel() // N
    dx = torch.empty_like(dy)
    dxd = torch.empty_like(dy) if drop is not None else None
    ctr, salt, p = drop if drop is not None else (None, 0, 0.0)
    nws = HIP.raw("kml_ln_bwd_ws_floats", M, N)
    ws = torch.empty(nws, dtype=F32, device=dy.device)
    cnt = _COUNTERS.take(dy.device, 1)
    if dbias_in is not None:
        _chk(dbias_in, F32, "dbias_in")
        if dbias_in.numel() < N:
            raise ValueError("dbias_in shorter than N")
    HIP.call("kml_ln_bwd", "p p p p p p p p p p p l i p p i f p s", _p(dy), _p(xin), _p(mean), _p(rstd), _p(gamma),
             _p(dx), _p(dx_add), _p(dgamma), _p(dbeta), _p(ws), _p(cnt), M, N, _p(dxd), _p(ctr),
             int(salt) & 0x7FFFFFFF, float(p), _p(dbias_in), _s())
    return (dx, dxd) if drop is not None else dx


def gelu_fwd(x):
    y = torch.empty_like(x)
    HIP.call("kml_gelu_fwd", "p p l s", _p(x), _p(y), x.numel(), _s())
    return y


def gelu_bwd(dy, x, dbias=None):
    """dx = dy * gelu'(x).  dbias (fp32 [N]) += column sums of dx over the rows of the
    [M, N] map, from the same pass (the bias gradient of the Linear whose pre-activation x is)."""
    dx = torch.empty_like(dy)
    if dbias is not None:
        _chk(dbias, F32, "dbias")
        N = dy.shape[-1]
        M = dy.numel() // N
        if dbias.numel() < N:
            raise ValueError("dbias shorter than N")
        ws = torch.empty(HIP.raw("kml_gelu_bwd_colsum_ws_floats", M, N), dtype=F32, device=dy.device)
        HIP.call("kml_gelu_bwd_colsum", "p p p p p l i s", _p(dy), _p(x), _p(dx), _p(dbias), _p(ws), M, N, _s())
        return dx
    HIP.call("kml_gelu_bwd", "p p p l s", _p(dy), _p(x), _p(dx), dy.numel(), _s())
    return dx


def dropout(x, ctr, salt, p):
    """Counter-based dropout: mask is a hash of (ctr[0] seed, ctr[1] step, salt, index)."""
    y = torch.empty_like(x)
    HIP.call("kml_dropout", "p p p i f l s", _p(x), _p(y), _p(ctr), int(salt) & 0x7FFFFFFF, float(p), x.numel(), _s())
    return y


def embed_fwd(ids, tt, word, pos, type_, L):
    T = ids.numel()
    N = word.shape[-1]
    out = torch.empty((T, N), dtype=BF16, device=ids.device)
    HIP.call("kml_embed_fwd", "p p p p p p l i i s", _p(ids), _p(tt), _p(word), _p(pos), _p(type_), _p(out), T, L, N,
             _s())
    return out


def embed_bwd(ids, tt, dsum, dword, dpos, dtype, L):
    """Word / position / token-type table gradients (+=).  With all three tables: one pass over
    dsum (k_embed_bwd_fused)."""
    T = ids.numel()
    N = dsum.shape[-1]
    HIP.call("kml_embed_bwd", "p p p p p p l i i s", _p(ids), _p(tt), _p(dsum), _p(dword), _p(dpos), _p(dtype), T, L,
             N, _s())


def gather_rows(src, idx):
    N = src.shape[-1]
    out = torch.empty((idx.numel(), N), dtype=src.dtype, device=src.device)
    HIP.call("kml_gather_rows", "p p p l i s", _p(src), _p(idx), _p(out), idx.numel(), N, _s())
    return out


def scatter_rows(src, idx, dst, accumulate=False):
    N = src.shape[-1]
    HIP.call("kml_scatter_rows", "p p p l i i s", _p(src), _p(idx), _p(dst), idx.numel(), N, int(accumulate), _s())
    return dst
