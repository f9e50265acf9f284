"""Launchers for the hand-written MFMA GEMM (csrc/kernels/gemm.hip).

``linear_fwd`` / ``linear_dgrad`` / ``linear_wgrad_`` are the three GEMMs of a linear
layer ``y = x W^T + b`` with bf16 activations, the bf16 weight shadow and the fp32
gradient storage of the flat parameter space.  Host-side checks guard every contract the
kernel relies on (alignment, multiples of 8/4) before a launch — a wrong shape never
reaches the GPU.  Tile and split-K choices come from a small per-shape table measured by
``tools/gemm_micro.py`` (``gemm_tuning.json``) with a heuristic default.
"""
from __future__ import annotations

import json
import os

import torch

from .._native import HIP, stream_ptr

BF16 = torch.bfloat16
F32 = torch.float32
TILES = {(256, 256): 0, (256, 128): 1, (128, 256): 2, (128, 128): 3, (128, 128, 2): 4, (256, 256, 4): 5,
         (256, 256, 8): 6, (256, 192, 8): 7,
         # tiles 3 / 4 on the 32x32x16 MFMA (layout 0 only): the measured alternative to 16x16x32
         (128, 128, 3, "mf32"): 8, (128, 128, 2, "mf32"): 9}  # (BM, BN[, stages])
_TUNE_FILE = os.environ.get("KUBEML_GEMM_TUNING_FILE") or \
    os.path.join(os.path.dirname(os.path.abspath(__file__)), "gemm_tuning.json")
_TUNED: dict = {}
if os.path.exists(_TUNE_FILE):   # KUBEML_GEMM_TUNING_FILE=none: every GEMM on its default tile
    with open(_TUNE_FILE) as f:
        for e in json.load(f).get("entries", []):
            _TUNED[(e["layout"], e["M"], e["N"], e["K"])] = (tuple(e["tile"]), int(e.get("splits", 1)))

# Every GEMM runs on the hand-written MFMA kernels of gemm.hip: the round-5 table still sent 11
# plain forward / dgrad BERT shapes to hipBLASLt; round 6 routes them to their best measured
# hand tile (profiles/r6/gemm/blas_shapes.jsonl: 0.83-0.96x the library on the 16384-token
# shapes, 1.4-1.7x on the MLM head's 2432-token ones).

_ZP = {}


ADD_C2 = 3  # kml_gemm act code: bf16 output = bf16(bf16(A B) + c2)


def _zp(dev):
    z = _ZP.get(dev)
    if z is None:
        z = torch.zeros(64, dtype=BF16, device=dev)
        _ZP[dev] = z
    return z


def _cdiv(a, b):
    return -(-a // b)


def _splits_for(tiles: int, K: int, min_chunk: int) -> int:
    """Smallest power of two s <= 8 with tiles * s >= 256 blocks (one per CU) while every
    split keeps >= min_chunk of the reduction."""
    s = 1
    while s < 8 and tiles * s < 256 and K // (2 * s) >= min_chunk:
        s *= 2
    return s


def plan(layout: int, M: int, N: int, K: int):
    """(tile, splits): the measured table (tools/gemm_bench.py), else the measured-best
    general choice — 128x128 two-stage tiles (two blocks per CU hide each other's
    prologue / epilogue), split-K when the output tiles cannot fill 256 CUs."""
    t = _TUNED.get((layout, M, N, K))
    if t is not None:
        return t
    tile = (128, 128, 2)
    tiles = _cdiv(M, 128) * _cdiv(N, 128)
    if layout == 2:
        return tile, _splits_for(tiles, K, 1024)
    if tiles < 128 and K >= 4096:
        return tile, _splits_for(tiles, K, 1024)
    return tile, 1


def _check(t, dtype, name):
    if t.dtype != dtype or not t.is_cuda:
        raise TypeError(f"{name}: expected CUDA {dtype}, got {t.dtype} on {t.device}")
    if t.data_ptr() % 16:
        raise ValueError(f"{name}: pointer must be 16-byte aligned")


def gemm(a, lda, b, ldb, c, ldc, M, N, K, layout, out, bias=None, act=0, c2=None, beta=0.0, tile=None,
         splits=None):
    """Raw launcher; see gemm.hip for the layout / out codes."""
    _check(a, BF16, "a")
    _check(b, BF16, "b")
    _check(c, BF16 if out == 0 else F32, "c")
    if N % 4 or ldc % 4:
        raise ValueError("gemm: N and ldc must be multiples of 4")
    if lda % 8 or ldb % 8:
        raise ValueError("gemm: leading dimensions must be multiples of 8")
    if K % 8:
        raise ValueError("gemm: K must be a multiple of 8")
    if bias is not None:
        _check(bias, F32, "bias")
        if bias.numel() < N:
            raise ValueError("gemm: bias shorter than N")
    if c2 is not None:
        _check(c2, BF16, "c2")
    if tile is None or splits is None:
        pt, ps = plan(layout, M, N, K)
        tile = tile or pt
        splits = splits or ps
    if out == 3:
        return wgrad_splitk_(c, a, lda, b, ldb, M, N, K, beta=beta, tile=tile, splits=splits)
    if out != 2:
        splits = 1
    if TILES[tuple(tile)] in (6, 7) and out == 0 and (N % 8 or ldc % 8):
        raise ValueError("gemm: the 256x256 phase tile with bf16 output needs N and ldc % 8 == 0")
    HIP.call("kml_gemm", "p l p l p l p p p i i i i i i f i i s", a.data_ptr(), int(lda), b.data_ptr(), int(ldb),
             c.data_ptr(), int(ldc), 0 if c2 is None else c2.data_ptr(), 0 if bias is None else bias.data_ptr(),
             _zp(a.device).data_ptr(), int(M), int(N), int(K), int(layout), int(out), int(act), float(beta),
             TILES[tuple(tile)], int(splits), stream_ptr())


def wgrad_splitk_(dw, a, lda, b, ldb, M, N, K, beta=1.0, tile=(256, 256, 8), splits=None):
    """dw[M][N] (fp32, contiguous) = beta * dw + A^T B with A [K][M], B [K][N] (layout 2):
    every K-slice stores its fp32 partial tile to a slab, one pass sums the slabs in order
    (deterministic, no atomics).  ``splits`` defaults to filling 256 CUs with one tile each."""
    _check(a, BF16, "a")
    _check(b, BF16, "b")
    _check(dw, F32, "dw")
    if not dw.is_contiguous() or dw.numel() != M * N:
        raise ValueError("wgrad_splitk_: dw must be a contiguous [M][N] fp32 tensor")
    if N % 4 or lda % 8 or ldb % 8:
        raise ValueError("wgrad_splitk_: N % 4 and leading dimensions % 8 must be 0")
    bm, bn = tile[0], tile[1]
    if splits is None:
        tiles = _cdiv(M, bm) * _cdiv(N, bn)
        splits = max(1, min(64, round(256 / tiles), K // 256))
    step = 64
    chunk = _cdiv(_cdiv(K, splits), step) * step
    nz = _cdiv(K, chunk)
    slab = torch.empty(nz * M * N, dtype=F32, device=dw.device)
    HIP.call("kml_gemm_wgrad_splitk", "p l p l p p p i i i f i i s", a.data_ptr(), int(lda), b.data_ptr(), int(ldb),
             dw.data_ptr(), slab.data_ptr(), _zp(a.device).data_ptr(), int(M), int(N), int(K), float(beta),
             TILES[tuple(tile)], int(splits), stream_ptr())
    return dw


def linear_fwd(x, w, bias=None, act=0, pre=None, bias16=None):
    """y[T, op] = act(x[T, ip] @ w[op, ip]^T + bias); ``pre`` receives the pre-activation.
    bias16: accepted for API compatibility (the MFMA epilogue adds the fp32 bias)."""
    T, ip = x.shape
    op = w.shape[0]
    if w.shape[1] != ip:
        raise ValueError(f"linear_fwd: x {tuple(x.shape)} vs w {tuple(w.shape)}")
    y = torch.empty((T, op), dtype=BF16, device=x.device)
    gemm(x, ip, w, ip, y, op, T, op, ip, 0, 0, bias=bias, act=act, c2=pre)
    return y


def linear_dgrad(dy, w, addend=None):
    """dx[T, ip] = dy[T, op] @ w[op, ip] (+ addend, a bf16 [T, ip] gradient summed in the
    epilogue exactly as a separate bf16 add would: the residual-gradient sum of a
    transformer layer, nn/transformer.py).  Few output tiles with a long reduction (the MLM
    decoder: 2432 x 768 out, K = 30528) split K over fp32 atomics into a scratch tile,
    then one bf16 conversion pass."""
    T, op = dy.shape
    ip = w.shape[1]
    if w.shape[0] != op:
        raise ValueError(f"linear_dgrad: dy {tuple(dy.shape)} vs w {tuple(w.shape)}")
    if addend is not None and (tuple(addend.shape) != (T, ip) or not addend.is_contiguous()):
        raise ValueError("linear_dgrad: addend must be a contiguous [T, ip] tensor")
    dx = torch.empty((T, ip), dtype=BF16, device=dy.device)
    tile, splits = plan(1, T, ip, op)
    if splits > 1:
        from . import kernels as KK
        acc = torch.empty((T, ip), dtype=F32, device=dy.device)
        KK.memset_(acc)
        gemm(dy, op, w, ip, acc, ip, T, ip, op, 1, 2, tile=tile, splits=splits)
        KK.f32_to_bf16(acc, dx)
        if addend is not None:
            KK.add_bf16(dx, addend, out=dx)
        return dx
    gemm(dy, op, w, ip, dx, ip, T, ip, op, 1, 0, tile=tile, splits=1, c2=addend,
         act=ADD_C2 if addend is not None else 0)
    return dx


def linear_dgrad_gelu(dy, w, pre, dbias=None):
    """dx = bf16(bf16(dy @ w) * gelu'(pre)) in the dgrad epilogue — the GELU backward of the
    layer whose output this linear consumed (FFN1 -> FFN2), and ``dbias`` (fp32) += column
    sums of dx (FFN1's bias gradient).  Only for shapes whose plan is the 256x256 phase tile
    without split-K; returns None otherwise (the caller runs the separate GELU backward)."""
    T, op = dy.shape
    ip = w.shape[1]
    tile, splits = plan(1, T, ip, op)
    if TILES.get(tuple(tile)) != 6 or splits != 1 or ip % 8 or tuple(pre.shape) != (T, ip):
        return None
    _check(dy, BF16, "dy")
    _check(w, BF16, "w")
    _check(pre, BF16, "pre")
    dx = torch.empty((T, ip), dtype=BF16, device=dy.device)
    colpart = torch.empty((_cdiv(T, 256), ip), dtype=F32, device=dy.device)
    HIP.call("kml_gemm_dgrad_gelu", "p l p l p l p p p i i i s", dy.data_ptr(), int(op), w.data_ptr(), int(ip),
             dx.data_ptr(), int(ip), pre.data_ptr(), colpart.data_ptr(), _zp(dy.device).data_ptr(), int(T), int(ip),
             int(op), stream_ptr())
    if dbias is not None:
        _check(dbias, F32, "dbias")
        HIP.call("kml_colreduce_add", "p i i p s", colpart.data_ptr(), int(colpart.shape[0]), int(ip),
                 dbias.data_ptr(), stream_ptr())
    return dx


def wgrad_can_store(op, ip, T) -> bool:
    """True if linear_wgrad_ for this shape can overwrite dw (slab split-K or a single pass:
    dw = 0 * dw + ...); False for the fp32-atomic split-K form, which only adds."""
    tile, splits = plan(2, op, ip, T)
    return len(tile) == 4 or splits <= 1


def linear_wgrad_(dw, dy, x, accumulate=True):
    """dw[op, ip] (fp32) += dy[T, op]^T @ x[T, ip]; ``accumulate=False`` overwrites dw (the
    first gradient write of a step: the region needs no zeroing, and the reduce never reads
    it) — only where :func:`wgrad_can_store`."""
    T, op = dy.shape
    ip = x.shape[1]
    if tuple(dw.shape) != (op, ip) or x.shape[0] != T:
        raise ValueError(f"linear_wgrad_: dw {tuple(dw.shape)} dy {tuple(dy.shape)} x {tuple(x.shape)}")
    if not dw.is_contiguous():
        raise ValueError("linear_wgrad_: dw must be contiguous")
    tile, splits = plan(2, op, ip, T)
    beta = 1.0 if accumulate else 0.0
    if len(tile) == 4:    # (BM, BN, stages, "slab"): deterministic slab split-K
        return wgrad_splitk_(dw, dy, op, x, ip, op, ip, T, beta=beta, tile=tile[:3], splits=splits)
    if splits > 1 and not accumulate:
        raise ValueError("linear_wgrad_: the atomic split-K form only accumulates")
    gemm(dy, op, x, ip, dw, ip, op, ip, T, 2, 2 if splits > 1 else 1, beta=beta, tile=tile, splits=splits)
    return dw
