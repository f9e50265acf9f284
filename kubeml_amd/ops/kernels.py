"""Thin, checked launchers for the HIP kernels in ``csrc/kernels``.

Every function here takes torch tensors that already live on an MI355X, validates
shape / dtype / contiguity on the host (a wrong shape must never reach a kernel),
allocates outputs from PyTorch's caching allocator and launches on PyTorch's
current stream — so the calls compose with ``torch.cuda.graph`` capture.

Tensor conventions
------------------
* activations: bf16, NHWC contiguous, C % 8 == 0
* conv weights: bf16 KRSC ``[Cout, KH, KW, Cin]`` contiguous (the bf16 shadow)
* weight gradients: fp32 KRSC, stored (``=``) or accumulated (``+=``) into the caller's buffer,
  one writer per element (no atomics: bitwise reproducible)
"""
from __future__ import annotations

import contextlib
import json
import math
import os

import torch

from .. import _native
from .._native import HIP

BF16 = torch.bfloat16
F32 = torch.float32


def _s() -> int:
    return _native.stream_ptr()


def _p(t) -> int:
    return 0 if t is None else t.data_ptr()


def _chk(t, dtype, name, ndim=None):
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_cuda:
        raise ValueError(f"{name}: must be a GPU tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if ndim is not None and t.dim() != ndim:
        raise ValueError(f"{name}: expected {ndim}-d tensor, got shape {tuple(t.shape)}")


# --------------------------------------------------------------------------------------
# convolution (implicit GEMM, MFMA)
# --------------------------------------------------------------------------------------

_TILES = [(128, 128), (128, 64), (64, 128), (64, 64), (64, 32), (32, 64), (32, 32)]
_TUNED: dict = {}  # (mode, M, N, Kd) -> (bm, bn, bk, splits); loaded from conv_tuning.json
_TUNED_PAIR: dict = {}  # (dgrad M, N, Kd, wgrad M, N, Kd) -> (dgrad plan, wgrad plan) of a grouped launch
_TUNE_FILE = os.environ.get("KUBEML_CONV_TUNING_FILE") or \
    os.path.join(os.path.dirname(os.path.abspath(__file__)), "conv_tuning.json")


def _load_tuning():
    # KUBEML_CONV_TUNING_FILE=none: every conv on its default plan
    if os.path.exists(_TUNE_FILE):
        with open(_TUNE_FILE) as f:
            for e in json.load(f).get("entries", []):
                if e["mode"] == "pair":
                    _TUNED_PAIR[(e["M"], e["N"], e["Kd"]) + tuple(e["wgrad"])] = (tuple(e["cfg"]), tuple(e["wcfg"]))
                else:
                    _TUNED[(e["mode"], e["M"], e["N"], e["Kd"])] = tuple(e["cfg"])


_load_tuning()


def out_hw(H, W, KH, KW, sh, sw, ph, pw):
    return (H + 2 * ph - KH) // sh + 1, (W + 2 * pw - KW) // sw + 1


def tap_window(H, W, KH, KW, sh, sw, ph, pw):
    """Taps [r0,r1)x[s0,s1) that touch the image for some output pixel (mirrors the C++)."""
    OH, OW = out_hw(H, W, KH, KW, sh, sw, ph, pw)

    def axis(I, O, K, st, p):
        ok = [t for t in range(K) if any(0 <= o * st - p + t < I for o in range(O))]
        return (ok[0], ok[-1] + 1) if ok else (0, 0)
    r0, r1 = axis(H, OH, KH, sh, ph)
    s0, s1 = axis(W, OW, KW, sw, pw)
    return r0, r1, s0, s1


def _cdiv(a, b):
    return -(-a // b)


def effective_splits(Kd, bk, splits):
    splits = max(1, splits)
    chunk = max(bk, _cdiv(_cdiv(Kd, splits), bk) * bk)
    return max(1, _cdiv(Kd, chunk))


def default_plan(mode, M, N, Kd, target_blocks=512):
    """Heuristic (bm, bn, bk, splits); tools/tune_conv.py measured tables override it."""
    bk = 64 if Kd >= 256 else 32
    best = None
    for bm, bn in [(64, 64), (128, 64), (64, 128), (128, 128), (64, 32), (32, 64), (32, 32)]:
        if bm > max(32, _cdiv(M, 32) * 32) or bn > max(32, _cdiv(N, 32) * 32):
            continue
        tiles = _cdiv(M, bm) * _cdiv(N, bn)
        kiters = _cdiv(Kd, bk)
        max_split = max(1, kiters // 4) if mode != "wgrad" else max(1, kiters // 8)
        if mode != "wgrad":
            max_split = min(max_split, 16)
        splits = max(1, min(max_split, round(target_blocks / tiles)))
        blocks = tiles * splits
        score = (min(blocks, target_blocks), bm * bn)
        if best is None or score > best[0]:
            best = (score, (bm, bn, bk, splits))
    return best[1] if best else (32, 32, 32, 1)


def plan_conv(mode, M, N, Kd):
    """(bm, bn, bk, splits, variant); variant 0 = register-staged pipeline,
    1/2 = LDS-DMA (global_load_lds) pipeline with 3/4 stages (BK fixed at 64),
    3 = direct LDS-free kernel (fwd/dgrad; bk = waves splitting K, splits = 1)."""
    cfg = _TUNED.get((mode, M, N, Kd))
    cfg = cfg if cfg is not None else default_plan(mode, M, N, Kd)
    return tuple(tuple(cfg) + (0,) * (5 - len(cfg)))


def _norm_cfg(cfg):
    bm, bn, bk, splits, variant = tuple(cfg) + (0,) * (5 - len(cfg))
    if variant in (1, 2):
        bk = 64  # the LDS-DMA pipeline is BK=64 only
    return bm, bn, bk, splits, variant


class _CounterPool:
    """Per-device pool of split-K ticket counters (zeroed once; kernels reset their own)."""

    SIZE = 1 << 16

    def __init__(self):
        self.bufs = {}
        self.pos = {}

    def take(self, device, n):
        buf = self.bufs.get(device)
        if buf is None:
            buf = torch.zeros(self.SIZE, dtype=torch.int32, device=device)
            self.bufs[device] = buf
            self.pos[device] = 0
        if n > self.SIZE:
            raise ValueError("too many split-K tiles")
        p = self.pos[device]
        if p + n > self.SIZE:
            p = 0
        self.pos[device] = p + n
        return buf[p:p + n]


_COUNTERS = _CounterPool()


def _splitk_ws(device, M, N, bm, bn, splits):
    if splits <= 1:
        return None, None
    tiles = _cdiv(M, bm) * _cdiv(N, bn)
    slab = torch.empty(tiles * splits * bm * bn, dtype=F32, device=device)
    return slab, _COUNTERS.take(device, tiles)


DIRECT = 3  # cfg variant id of the LDS-free wave-split-K kernel (fwd / dgrad)


# Partial BN rows above this count are group-reduced inside the producing conv (the last
# block of every group of M-tiles sums its group's rows): the consumer BN kernel, whose every
# block otherwise re-reads all rows from L2, then reads at most 16 rows.  Off (0) for plain
# consumers: on ResNet-34/b256 the ticket hand-off in every producer block costs more than the
# consumer saves (1.720 ms/step off vs 1.758-1.782 at 64..512 rows); consumers whose every block
# reads all rows ask for it (``group=True``).
_GRP_MIN = 0
_GRP_ROWS = 16




def _stats_layout(M, cfg, group=False):
    """(per-wave rows G, M-tiles per group or 0, rows the consumer reads).  group: reduce
    to at most _GRP_ROWS rows regardless of _GRP_MIN (a consumer whose every block reads all
    rows, e.g. the BN-folding halo conv)."""
    bm = _norm_cfg(cfg)[0]
    tiles = _cdiv(M, bm)
    # one row per M tile (the epilogue sums the tile's wave row-bands; tail tiles included)
    G = tiles
    if group:
        if G <= _GRP_ROWS:
            return G, 0, G
    elif _GRP_MIN <= 0 or G <= _GRP_MIN:
        return G, 0, G
    tpg = _cdiv(tiles, _GRP_ROWS)
    return G, tpg, _cdiv(tiles, tpg)


def conv_stats_rows(M, cfg, group=False):
    """Rows of the partial-statistics buffer a conv epilogue hands to the BN kernel for a
    plan: one per M-tile, or one per M-tile group when group-reduced."""
    return _stats_layout(M, cfg, group)[2]


def _stats_ws(device, M, N, cfg, out, group=False):
    """(rows buffer the epilogue writes, group output or None, tickets, tiles per group)."""
    G, tpg, ng = _stats_layout(M, cfg, group)
    if not tpg:
        return out, None, None, 0
    bn = _norm_cfg(cfg)[1]
    scratch = torch.empty(G * 2 * N, dtype=F32, device=device)
    return scratch, out, _COUNTERS.take(device, ng * _cdiv(N, bn)), tpg


def unrolled22(H, W, KH, KW, stride, pad) -> bool:
    """True for the convs that run unrolled: 3x3 / stride 1 / pad 1 on a 2x2 map.

    There every output pixel sees only 4 of the 9 taps (the other 5 read padding), so
    the conv is the dense map [B, 4C] -> [B, 4K] of the NHWC rows with the gathered weight
    wu[(p, n)][(q, c)] = w[n][tap(p, q)][c] (:func:`unroll22_multi`): a 1x1 conv with 4/9 of
    the im2col FLOPs (ResNet-34/18 layer3 at 32x32 input, 2x2 maps).  BN statistics fold the
    4 positions back onto the K channels in the epilogue (``fold_c``) and the weight
    gradient scatters back onto the 3x3 taps (``u_k0/u_c0``)."""
    return (H, W, KH, KW) == (2, 2, 3, 3) and tuple(stride) == (1, 1) and tuple(pad) == (1, 1)


def unroll22_multi(ws, wus):
    """wus[i][4K,1,1,4C] = unrolled form of ws[i][K,3,3,C] for up to 16 convs, one launch."""
    import ctypes
    n = len(ws)
    if n == 0:
        return
    if n > 16 or len(wus) != n:
        raise ValueError("unroll22_multi: 1..16 pairs")
    wp = (ctypes.c_void_p * n)()
    up = (ctypes.c_void_p * n)()
    dims = (ctypes.c_int * (2 * n))()
    for i, (w, wu) in enumerate(zip(ws, wus)):
        _chk(w, BF16, "w", 4)
        _chk(wu, BF16, "wu", 4)
        K, KH, KW, C = w.shape
        if (KH, KW) != (3, 3) or tuple(wu.shape) != (4 * K, 1, 1, 4 * C) or C % 8:
            raise ValueError("unrolled weight shape mismatch")
        wp[i], up[i] = w.data_ptr(), wu.data_ptr()
        dims[2 * i], dims[2 * i + 1] = K, C
    HIP.call("kml_conv_unroll22_multi", "p p p i s", ctypes.addressof(wp), ctypes.addressof(up),
             ctypes.addressof(dims), n, _s())


def unrolled_weight(w, out=None):
    """The [4K,1,1,4C] unrolled weight of a 3x3 conv (one launch)."""
    K, KH, KW, C = w.shape
    if out is None:
        out = torch.empty((4 * K, 1, 1, 4 * C), dtype=BF16, device=w.device)
    unroll22_multi([w], [out])
    return out


def unroll22_reference(w):
    """Plain-PyTorch form of the unrolled weight (any device/dtype; the kernel's mapping):
    wu[(p, n)][(q, c)] = w[n][qh - ph + 1][qw - pw + 1][c] for positions p, q of a 2x2 map."""
    K, KH, KW, C = w.shape
    wu = w.new_zeros((4, K, 4, C))
    for p in range(4):
        for q in range(4):
            r, s = (q >> 1) - (p >> 1) + 1, (q & 1) - (p & 1) + 1
            wu[p, :, q, :] = w[:, r, s, :]
    return wu.reshape(4 * K, 1, 1, 4 * C)


class _Gather22:
    """``wu=GATHER22``: run an unrolled conv in its 1x1 form WITHOUT a materialised unrolled
    weight — the FWD / DGRAD weight loaders gather W'[(p, n)][(q, c)] = w[n][tap(p, q)][c]
    straight from the 3x3 weight (no k_unroll22_multi pass per step).  Not for the direct
    (transposed-weight) dgrad variant."""

    def __repr__(self):
        return "GATHER22"


GATHER22 = _Gather22()


def _g22_weight_ok(w, K1, C1):
    """The 3x3 weight of a gathered 1x1-form conv of K1 = 4K outputs, C1 = 4C inputs."""
    return tuple(w.shape) == (K1 // 4, 3, 3, C1 // 4) and K1 % 4 == 0 and C1 % 32 == 0


def _check_wu(x_shape, w, wu, KH, KW, stride, pad):
    B, H, W, C = x_shape
    if not unrolled22(H, W, KH, KW, stride, pad):
        raise ValueError("wu given for a conv that is not unrolled (3x3/s1/p1 on 2x2)")
    K = w.shape[0]
    if wu is GATHER22:
        if C % 8:
            raise ValueError("gathered unrolled conv: Cin must be a multiple of 8")
        return B, C, K
    _chk(wu, BF16, "wu", 4)
    if tuple(wu.shape) != (4 * K, 1, 1, 4 * C):
        raise ValueError(f"unrolled weight shape {tuple(wu.shape)} != {(4 * K, 1, 1, 4 * C)}")
    return B, C, K


def conv_fwd(x, w, KH, KW, stride, pad, bias=None, stats=None, relu=False, out=None, cfg=None, stats_part=False,
             wu=None, _fold=0, _g22=False, stats_group=False):
    """y[B,OH,OW,Cout] = conv(x[B,H,W,Cin], w[Cout,KH,KW,Cin]) (+bias, ReLU; BN stats).

    stats: fp32 [2*Cout] accumulated with atomics, or with ``stats_part`` a [G, 2*Cout]
    buffer of per-wave partial rows (``G = conv_stats_rows(M, plan)``, see
    :func:`conv_fwd_plan`) that :func:`bn_apply` sums — no zeroing, no atomics.
    wu: unrolled weight (:func:`unrolled22`): the conv runs as its dense 1x1 form
    (``GATHER22``: gathered from ``w`` by the kernel)."""
    _chk(x, BF16, "x", 4)
    _chk(w, BF16, "w", 4)
    if wu is not None:
        B, C, K = _check_wu(x.shape, w, wu, KH, KW, stride, pad)
        if stats is not None and not stats_part:
            raise ValueError("unrolled conv: BN statistics need stats_part")
        if out is not None and tuple(out.shape) != (B, 2, 2, K):
            raise ValueError("out shape mismatch")
        o = None if out is None else out.view(B, 1, 1, 4 * K)
        g = wu is GATHER22
        y = conv_fwd(x.view(B, 1, 1, 4 * C), w if g else wu, 1, 1, (1, 1), (0, 0), bias=bias, stats=stats, relu=relu,
                     out=o, cfg=cfg, stats_part=stats_part, _fold=K, _g22=g)
        return y.view(B, 2, 2, K)
    B, H, W, C = x.shape
    K = 4 * w.shape[0] if _g22 else w.shape[0]
    if _g22:
        if (KH, KW) != (1, 1) or not _g22_weight_ok(w, K, C):
            raise ValueError(f"gathered unrolled weight {tuple(w.shape)} does not match the 1x1 form {K}x{C}")
    elif tuple(w.shape[1:]) != (KH, KW, C):
        raise ValueError(f"weight shape {tuple(w.shape)} does not match KH={KH} KW={KW} Cin={C}")
    if C % 8:
        raise ValueError("Cin must be a multiple of 8 (pad channels)")
    sh, sw = stride
    ph, pw = pad
    OH, OW = out_hw(H, W, KH, KW, sh, sw, ph, pw)
    if out is None:
        out = torch.empty((B, OH, OW, K), dtype=BF16, device=x.device)
    if bias is not None:
        _chk(bias, F32, "bias")
        assert bias.numel() >= K
    r0, r1, s0, s1 = tap_window(H, W, KH, KW, sh, sw, ph, pw)
    M, Kd = B * OH * OW, (r1 - r0) * (s1 - s0) * C
    bm, bn, bk, splits, variant = conv_fwd_plan(C, M, K, Kd, cfg, geom=(H, W, KH, KW, stride, pad))
    rows, grp, gcnt, tpg = stats, None, None, 0
    if stats is not None:
        _chk(stats, F32, "stats")
        need = 2 * K * (conv_stats_rows(M, (bm, bn, bk, splits, variant), stats_group) if stats_part else 1)
        if _fold and (not stats_part or K % _fold):
            raise ValueError("folded statistics need stats_part and K % fold == 0")
        if stats.numel() < need:
            raise ValueError(f"stats buffer has {stats.numel()} floats, needs {need}")
        if stats_part:
            rows, grp, gcnt, tpg = _stats_ws(x.device, M, K, (bm, bn, bk, splits, variant), stats, stats_group)
    if _fold and grp is not None:
        raise ValueError("folded statistics cannot be group-reduced")
    sig = "p p p p p i i i i i i i i i i i i i i i i i i p p p p i i i s"
    if variant == HALO:
        HIP.call("kml_conv_fwd", sig, _p(x), _p(w), _p(out), _p(bias), _p(rows), int(stats_part), B, H, W, C, K,
                 KH, KW, sh, sw, ph, pw, int(relu), bm, bn, 0, 1, HALO, 0, 0, _p(grp), _p(gcnt), tpg, 0, 0, _s())
        return out
    if variant == STEM:
        HIP.call("kml_conv_fwd", sig, _p(x), _p(w), _p(out), _p(bias), _p(rows), int(stats_part), B, H, W, C, K,
                 KH, KW, sh, sw, ph, pw, int(relu), bm, bn, 0, 1, STEM, 0, 0, _p(grp), _p(gcnt), tpg, 0, 0, _s())
        return out
    if variant == ONESHOT:
        HIP.call("kml_conv_fwd", sig, _p(x), _p(w), _p(out), _p(bias), _p(rows), int(stats_part), B, H, W, C, K,
                 KH, KW, sh, sw, ph, pw, int(relu), bm, bn, 0, 1, ONESHOT, 0, 0, _p(grp), _p(gcnt), tpg,
                 int(_fold), int(_g22), _s())
        return out
    if variant == GEMM1X1:
        if relu or _fold or _g22 or grp is not None or (stats is not None and not stats_part) or \
                not x.is_contiguous() or not out.is_contiguous():
            # same bm (and the same row grouping), so the statistics rows the caller sized stay valid
            return conv_fwd(x, w, KH, KW, stride, pad, bias=bias, stats=stats, relu=relu, out=out,
                            cfg=_GEMM1X1_FALLBACK[bm], stats_part=stats_part, _fold=_fold, _g22=_g22,
                            stats_group=stats_group)
        from . import gemm as G
        zp = G._zp(x.device)
        if not gemm1x1_ok(C, K, H, W, KH, KW, stride, pad):   # implicit GEMM: A gathered per K-tile
            HIP.call("kml_gemm_conv_fwd", "p p p p p p i i i i i i i i i i i i p p i s", _p(x), _p(w), _p(out),
                     _p(bias), _p(rows), _p(zp), B, H, W, C, K, KH, KW, sh, sw, ph, pw, bk, _p(grp), _p(gcnt), tpg,
                     _s())
            return out
        if stats is None:
            HIP.call("kml_gemm", "p l p l p l p p p i i i i i i f i i s", _p(x), C, _p(w), C, _p(out), K, 0,
                     _p(bias), _p(zp), M, K, C, 0, 0, 0, 0.0, bk, 1, _s())
        else:
            HIP.call("kml_gemm_stats", "p l p l p l p p p i i i i p p i s", _p(x), C, _p(w), C, _p(out), K, _p(bias),
                     _p(rows), _p(zp), M, K, C, bk, _p(grp), _p(gcnt), tpg, _s())
        return out
    if variant == DIRECT:  # bk carries the wave count of the direct kernel
        _conv_fwd_launch(sig, (_p(x), _p(w), _p(out), _p(bias), _p(rows), int(stats_part), B, H, W, C, K,
                               KH, KW, sh, sw, ph, pw, int(relu), bm, bn, bk, 1, DIRECT, 0, 0, _p(grp), _p(gcnt), tpg,
                               int(_fold), int(_g22)), keep=(x, w, out, bias, rows, grp, gcnt))
        return out
    splits = effective_splits(Kd, bk, splits)
    slab, cnt = _splitk_ws(x.device, M, K, bm, bn, splits)
    _conv_fwd_launch(sig, (_p(x), _p(w), _p(out), _p(bias), _p(rows), int(stats_part), B, H, W, C, K, KH, KW,
                           sh, sw, ph, pw, int(relu), bm, bn, bk, splits, variant, _p(slab), _p(cnt), _p(grp), _p(gcnt),
                           tpg, int(_fold), int(_g22)), keep=(x, w, out, bias, rows, grp, gcnt, slab, cnt))
    return out


_FWD_PAIR = None   # list while a conv_fwd_pair() block records
FWD_PAIRS_LAUNCHED = [0]   # k_conv_fwd_pair launches so far (tests check the pair path ran)


def _conv_fwd_launch(sig, args, keep=()):
    """keep: every tensor the launch reads or writes.  A recorded launch runs later, so the record
    holds them: a workspace the caller drops (the group-reduction scratch rows) must not go back to
    the caching allocator — and to the other conv of the pair — before the kernel is launched."""
    if _FWD_PAIR is not None and len(_FWD_PAIR) < 2:
        _FWD_PAIR.append((sig, args, keep))
        return
    HIP.call("kml_conv_fwd", sig, *args, _s())


@contextlib.contextmanager
def conv_fwd_pair():
    """Launch the (up to) two conv_fwd calls made inside this block as ONE kernel when their plans
    form an instantiated forward pair (conv_igemm.hip k_conv_fwd_pair: the strided 3x3 and the
    1x1 projection of a downsampling residual block, which both read the block input); otherwise
    each launches on its own at the end of the block.  Only the register-staged / LDS-DMA / direct
    plans record; any other route launches immediately, as always.  The convs must not depend on
    each other."""
    global _FWD_PAIR
    prev, _FWD_PAIR = _FWD_PAIR, []
    try:
        yield
    finally:
        rec, _FWD_PAIR = _FWD_PAIR, prev
        rc = 1
        if len(rec) == 2:
            import ctypes
            q = [(ctypes.c_longlong * 30)(*[int(v) for v in a]) for _, a, _ in rec]
            rc = HIP.fn("kml_conv_fwd_pair", "p p s")(ctypes.addressof(q[0]), ctypes.addressof(q[1]), _s())
        if rc == 1:
            for sig, a, _ in rec:
                HIP.call("kml_conv_fwd", sig, *a, _s())
        elif rc:
            raise RuntimeError(f"kml_conv_fwd_pair failed: {rc}")
        else:
            FWD_PAIRS_LAUNCHED[0] += 1


def conv_fwd_plan(C, M, K, Kd, cfg=None, geom=None):
    """The (bm, bn, bk, splits, variant) conv_fwd will run for this shape.  ``geom`` =
    (H, W, KH, KW, stride, pad) lets an eligible conv take the halo-patch kernel
    (:func:`halo_plan`); without it (or when ineligible) a HALO plan falls back."""
    if cfg is None and geom is not None:
        OH, OW = out_hw(geom[0], geom[1], geom[2], geom[3], geom[4][0], geom[4][1], geom[5][0], geom[5][1])
        B = M // max(OH * OW, 1)
        hp = halo_plan(C, K, *geom) or oneshot_plan(C, K, Kd, *geom, B=B) or stem_plan(C, K, *geom)
        if hp is not None:
            return hp
    plan = _norm_cfg(cfg or plan_conv("fwd", M, K, Kd))
    if plan[4] == HALO and (geom is None or not halo_ok(C, K, *geom, plan[0], plan[1])):
        plan = _norm_cfg(default_plan("fwd", M, K, Kd))
    if plan[4] == ONESHOT and (geom is None or not oneshot_ok(C, K, Kd, *geom, plan[0], plan[1])):
        plan = _norm_cfg(default_plan("fwd", M, K, Kd))
    if plan[4] == STEM and (geom is None or stem_plan(C, K, *geom, force=True) is None):
        plan = _norm_cfg(default_plan("fwd", M, K, Kd))
    if plan[4] == DIRECT and C % 32:
        plan = _norm_cfg(default_plan("fwd", M, K, Kd))
    if plan[4] == GEMM1X1 and (geom is None or (plan[0], plan[1], plan[2]) not in _GEMM1X1_TILES or
                               not (gemm1x1_ok(C, K, *geom) or (plan[2] <= 4 and gemm_conv_ok(C, K, *geom)))):
        plan = _norm_cfg(default_plan("fwd", M, K, Kd))
    return plan


HALO = 4  # cfg variant id of the halo-patch forward (3x3/s1/p1 on small maps): bm = pixels, bn = channels
# (C, H) -> (bm, bn): the halo tiles the kernel is instantiated for, first = default
_HALO_TILES = {(64, 8): [(64, 32), (64, 64), (128, 64)],
               (128, 4): [(64, 32), (64, 64), (128, 32), (64, 128), (128, 64)],
               (256, 8): [(64, 64), (64, 32)], (256, 4): [(64, 32), (64, 64)],
               (512, 4): [(64, 32), (64, 64)]}


def halo_ok(C, K, H, W, KH, KW, stride, pad, bm, bn) -> bool:
    """Is (bm, bn) an instantiated halo tile for this conv?"""
    return ((KH, KW) == (3, 3) and tuple(stride) == (1, 1) and tuple(pad) == (1, 1) and H == W and
            (bm, bn) in _HALO_TILES.get((C, H), ()) and K % bn == 0)


# dgrad halo tiles, keyed by (Cout = the dy patch's channels, H): (bm, bn) with bn over Cin
_HALO_DG_TILES = {(64, 8): [(64, 32), (64, 64), (128, 64)], (128, 4): [(64, 32)]}
_HALO_DG_ON = False   # tests / micro-benchmarks only: measured slower in the step (profiles/r3/halo_dgrad.md)


def halo_dgrad_ok(C, K, H, W, KH, KW, stride, pad, bm, bn) -> bool:
    """Is (bm, bn) an instantiated halo dgrad tile for this conv (C = Cin, K = Cout)?"""
    return ((KH, KW) == (3, 3) and tuple(stride) == (1, 1) and tuple(pad) == (1, 1) and H == W and
            (bm, bn) in _HALO_DG_TILES.get((K, H), ()) and C % bn == 0)


def halo_dgrad_plan(C, K, H, W, KH, KW, stride, pad):
    """Halo-patch dgrad plan (patch of dy, flipped-filter weight slice in LDS) for an eligible
    conv when ``_HALO_DG_ON``, else None."""
    if not _HALO_DG_ON:
        return None
    for bm, bn in _HALO_DG_TILES.get((K, H), ()):
        if halo_dgrad_ok(C, K, H, W, KH, KW, stride, pad, bm, bn):
            return (bm, bn, K * 16 + H, 1, HALO)   # bk slot: the body's geometry (grouped pairs)
    return None


STEM = 6  # cfg variant id of the stem patch kernel (7x7/s2/p3, Cin 8, Cout 64; 32x32 or 224x224 input)
def stem_plan(C, K, H, W, KH, KW, stride, pad, force=False):
    """The ResNet ImageNet stem (7x7/s2/p3, Cin padded to 8, 64 out) as the patch-in-LDS
    kernel: (256, 64, 0, 1, STEM) on 32x32 images (one image per block), (224, 64, 0, 1,
    STEM) on 224x224 (persistent blocks over output row pairs, bm = 2 output rows), else None."""
    if (C, K, KH, KW, tuple(stride), tuple(pad)) != (8, 64, 7, 7, (2, 2), (3, 3)) or H != W:
        return None
    if H == 32:
        return (256, 64, 0, 1, STEM)
    if H == 224:
        return (224, 64, 0, 1, STEM)
    return None


ONESHOT = 5  # cfg variant id of the one-shot panel forward (single-tap convs, K in _ONESHOT_TILES)
_ONESHOT_TILES = {512: [(32, 32), (32, 64), (64, 32)], 1024: [(32, 32)], 256: [(32, 32), (32, 64), (64, 64)]}


GEMM1X1 = 7  # cfg variant id of the GEMM route: a 1x1 / stride-1 conv on the MFMA GEMM (gemm.hip)
# (bm, bn) -> gemm.hip tile code of the GEMM route (cfg = (bm, bn, tile, 1, GEMM1X1)); BN statistics
# come out of the GEMM's epilogue as one [sum | sumsq] row per bm rows (kml_gemm_stats)
_GEMM1X1_TILES = {(256, 256, 6), (256, 256, 0), (256, 128, 1), (128, 256, 2), (128, 128, 3), (128, 128, 4)}
# same-G implicit-GEMM stand-ins when a call cannot take the GEMM route (ReLU epilogue, grouped rows)
_GEMM1X1_FALLBACK = {128: (128, 64, 32, 1, 0), 256: (256, 128, 64, 1, 1)}


def gemm1x1_ok(C, K, H, W, KH, KW, stride, pad) -> bool:
    """Can this forward conv run as a plain GEMM x[M, C] @ w[K, C]^T (1x1, stride 1, no padding)?"""
    return (KH, KW) == (1, 1) and tuple(stride) == (1, 1) and tuple(pad) == (0, 0) and C % 8 == 0 and K % 8 == 0


def gemm_dgrad_gather_ok(C, K, stride) -> bool:
    """Can this conv's input gradient run on the GEMM tiles as an implicit GEMM (kml_gemm_conv_dgrad:
    stride 1, one filter tap per K-tile of dy's channels)?"""
    return tuple(stride) == (1, 1) and K % 64 == 0 and C % 8 == 0


def gemm_conv_ok(C, K, H, W, KH, KW, stride, pad) -> bool:
    """Can this forward conv run on the GEMM tiles as an implicit GEMM (kml_gemm_conv_fwd: the A
    operand gathered from x per K-tile, one filter tap per tile)?"""
    return C % 64 == 0 and K % 8 == 0


def oneshot_ok(C, K, Kd, H, W, KH, KW, stride, pad, bm, bn) -> bool:
    """Single-tap forward with contiguous A rows and an instantiated (bm, bn, Kd) panel pair."""
    if Kd != C or (bm, bn) not in _ONESHOT_TILES.get(Kd, ()):
        return False
    r0, r1, s0, s1 = tap_window(H, W, KH, KW, stride[0], stride[1], pad[0], pad[1])
    OH, OW = out_hw(H, W, KH, KW, stride[0], stride[1], pad[0], pad[1])
    rows = (H * W == 1 and OH * OW == 1) or ((KH, KW) == (1, 1) and tuple(stride) == (1, 1) and tuple(pad) == (0, 0))
    return (r1 - r0) == 1 and (s1 - s0) == 1 and rows


# Large maps take the tuned implicit GEMM instead: the one-shot panels (one block per CU at
# K = 1024, 32x32 tiles) run ResNet-50's 14x14 / 28x28 1x1 convs at ~95-135 TF/s against
# 290-380 for the tuned tiles, and at K = 256 the 128x64 tile now wins too (56x56 256->64:
# 55.9 vs 79.0 us, 14x14 256->1024: 51.9 vs 71.9 us; profiles/r5/r50_1x1_fwd.md).  The panels
# keep the small-M layers (1x1 maps, B rows).
_ONESHOT_MAX_ROWS = 4096


def oneshot_plan(C, K, Kd, H, W, KH, KW, stride, pad, B=0):
    """Default one-shot panel plan for an eligible forward conv, or None."""
    if B * H * W > _ONESHOT_MAX_ROWS:
        return None
    for bm, bn in _ONESHOT_TILES.get(Kd, ()):
        if oneshot_ok(C, K, Kd, H, W, KH, KW, stride, pad, bm, bn):
            return (bm, bn, 0, 1, ONESHOT)
    return None


# tests / micro-benchmarks only: as two launches the one-shot dgrad + wgrad lose to the grouped
# implicit-GEMM pair (1.376 vs 1.353 ms/step, profiles/r3/oneshot.md)
_ONESHOT_BWD_ON = False
_ONESHOT_DG_TILES = {1024: (32, 32), 512: (32, 32)}   # keyed by the dgrad K (= Cout)
_ONESHOT_WG_TILES = {256: (32, 32)}                    # keyed by the wgrad K (= pixels)


def oneshot_bwd_plans(C, K, B, H, W, KH, KW, stride, pad):
    """(dgrad plan or None, wgrad plan or None) of the one-shot backward bodies for a
    single-tap conv with contiguous rows (only when ``_ONESHOT_BWD_ON``)."""
    if not _ONESHOT_BWD_ON or C % 32 or K % 32:
        return None, None
    r0, r1, s0, s1 = tap_window(H, W, KH, KW, stride[0], stride[1], pad[0], pad[1])
    OH, OW = out_hw(H, W, KH, KW, stride[0], stride[1], pad[0], pad[1])
    rows = (H * W == 1 and OH * OW == 1) or ((KH, KW) == (1, 1) and tuple(stride) == (1, 1) and tuple(pad) == (0, 0))
    if not ((r1 - r0) == 1 and (s1 - s0) == 1 and rows):
        return None, None
    d = _ONESHOT_DG_TILES.get(K)
    w = _ONESHOT_WG_TILES.get(B * OH * OW)
    return ((d[0], d[1], 0, 1, ONESHOT) if d else None), ((w[0], w[1], 0, 1, ONESHOT) if w else None)


def halo_plan(C, K, H, W, KH, KW, stride, pad):
    """Default halo-patch plan for an eligible forward conv, or None."""
    for bm, bn in _HALO_TILES.get((C, H), ()):
        if halo_ok(C, K, H, W, KH, KW, stride, pad, bm, bn):
            return (bm, bn, 0, 1, HALO)
    return None


def conv_fwd_stats_rows(x_shape, K, KH, KW, stride, pad, cfg=None, unroll=False, group=False):
    """G of the partial-statistics buffer conv_fwd(stats_part=True) needs for this conv
    (``unroll``: the conv runs with its unrolled weight, 4 folded rows per M-tile)."""
    B, H, W, C = x_shape
    if unroll:
        if not unrolled22(H, W, KH, KW, stride, pad):
            raise ValueError("conv is not unrolled")
        return 4 * conv_stats_rows(B, conv_fwd_plan(4 * C, B, 4 * K, 4 * C, cfg, geom=(1, 1, 1, 1, (1, 1), (0, 0))))
    OH, OW = out_hw(H, W, KH, KW, stride[0], stride[1], pad[0], pad[1])
    r0, r1, s0, s1 = tap_window(H, W, KH, KW, stride[0], stride[1], pad[0], pad[1])
    M, Kd = B * OH * OW, (r1 - r0) * (s1 - s0) * C
    return conv_stats_rows(M, conv_fwd_plan(C, M, K, Kd, cfg, geom=(H, W, KH, KW, stride, pad)), group)


def bnin_ok(x_shape, K, KH, KW, stride, pad) -> bool:
    """Can this forward conv apply its input's BatchNorm + ReLU while staging (conv_fwd_bnin)?
    The halo kernel (3x3/s1/p1 on 8x8 / 4x4 maps).  The one-shot panels' BN-in form (layers 3-4)
    measured slower than the separate BN apply and was removed (profiles/r5/bn_fold_ab.md,
    profiles/r6/bn_final_rows.md)."""
    B, H, W, C = x_shape
    if not _BNIN_ON:
        return False
    if halo_plan(C, K, H, W, KH, KW, stride, pad) is not None:
        return 2 * C <= 1024 and 256 % (C // 2) == 0
    return False


def bnin_stats_rows(x_shape, K):
    """G of the output statistics rows of conv_fwd_bnin on an input of x_shape (3x3/s1/p1)."""
    return conv_fwd_stats_rows(x_shape, K, 3, 3, (1, 1), (1, 1))


_BNIN_ON = True


def conv_fwd_bnin(c_in, w, rows, G, gamma, beta, save_mean, save_rstd, run_mean, run_var, eps, momentum, y_in,
                  stats=None, stats_part=True, stats_group=False, out=None, res=None):
    """out = conv3x3(relu(bn(c_in))) on the halo kernel with the BatchNorm applied while the patch
    is staged: ``rows``/``G`` are the producer's partial statistics rows, the normalised input is
    written to ``y_in`` (every element, by the N-tile-0 blocks), ``save_mean``/``save_rstd`` and
    the running buffers are updated as bn_apply would.  ``stats`` as in :func:`conv_fwd` (the
    output's own BN partial rows).  res: the folded BN's residual, y_in = relu(bn(c_in) + res)
    (a block's output BN applied by the next block's first conv)."""
    _chk(c_in, BF16, "c_in", 4)
    _chk(w, BF16, "w", 4)
    _chk(y_in, BF16, "y_in", 4)
    if res is not None:
        _chk(res, BF16, "res", 4)
        if tuple(res.shape) != tuple(c_in.shape):
            raise ValueError("conv_fwd_bnin: residual shape must match c_in")
    B, H, W, C = c_in.shape
    K = w.shape[0]
    if tuple(w.shape) != (K, 3, 3, C) or tuple(y_in.shape) != tuple(c_in.shape):
        raise ValueError("conv_fwd_bnin: 3x3 weight over c_in's channels and a y_in like c_in")
    plan = halo_plan(C, K, H, W, 3, 3, (1, 1), (1, 1))
    if plan is None or not bnin_ok(c_in.shape, K, 3, 3, (1, 1), (1, 1)):
        raise ValueError("conv_fwd_bnin: conv is not halo-eligible")
    bm, bn = plan[0], plan[1]
    if out is None:
        out = torch.empty((B, H, W, K), dtype=BF16, device=c_in.device)
    srows, grp, gcnt, tpg = stats, None, None, 0
    if stats is not None:
        _chk(stats, F32, "stats")
        need = 2 * K * (conv_stats_rows(B * H * W, plan, stats_group) if stats_part else 1)
        if stats.numel() < need:
            raise ValueError(f"stats buffer has {stats.numel()} floats, needs {need}")
        if stats_part:
            srows, grp, gcnt, tpg = _stats_ws(c_in.device, B * H * W, K, plan, stats, stats_group)
    _chk(rows, F32, "rows")
    if rows.numel() < G * 2 * C:
        raise ValueError("conv_fwd_bnin: partial rows smaller than G x 2C")
    HIP.call("kml_conv_fwd_bnin", "p p p p i i i i i i i i p p i p i p p p p p p f f p p s",
             _p(c_in), _p(w), _p(out), _p(srows), int(stats_part), B, H, W, C, K, bm, bn, _p(grp), _p(gcnt), tpg,
             _p(rows), int(G), _p(gamma), _p(beta), _p(save_mean), _p(save_rstd), _p(run_mean), _p(run_var),
             float(eps), float(momentum), _p(y_in), _p(res), _s())
    return out


def _u22_views(B, C, K, dy=None, x=None, addend=None, bnf=None):
    """Views of the NHWC [B,2,2,*] tensors of an unrolled conv as its 1x1 form [B,1,1,4*]."""
    v = lambda t, n: None if t is None else t.reshape(B, 1, 1, 4 * n)
    b = None if bnf is None else (v(bnf[0], C), v(bnf[1], C), bnf[2], bnf[3])
    return v(dy, K), v(x, C), v(addend, C), b


def conv_dgrad(dy, w, in_shape, KH, KW, stride, pad, out=None, addend=None, cfg=None, bnf=None, wt=None, wu=None,
               _fold=0, bnf_mask=False, _g22=False):
    """dx = conv input gradient (+ addend, the fused residual-gradient sum).

    bnf = (y or None, c, mean, rstd) of the BatchNorm that consumes dx: the epilogue also
    writes that BN's dgamma/dbeta partial rows; returns (dx, (part, G)) for
    :func:`bn_bwd(partial=...)`.  bnf_mask: return dz = dx * [y > 0] instead (the consumer's
    ReLU mask applied here, so its bn_bwd runs with y=None and never reads y).
    wu: unrolled weight (:func:`unrolled22`)."""
    _chk(dy, BF16, "dy", 4)
    _chk(w, BF16, "w", 4)
    if wu is not None:
        B, C, K = _check_wu(in_shape, w, wu, KH, KW, stride, pad)
        dy1, _, add1, bnf1 = _u22_views(B, C, K, dy=dy, addend=addend, bnf=bnf)
        o = None if out is None else out.view(B, 1, 1, 4 * C)
        g = wu is GATHER22
        r = conv_dgrad(dy1, w if g else wu, (B, 1, 1, 4 * C), 1, 1, (1, 1), (0, 0), out=o, addend=add1, cfg=cfg,
                       bnf=bnf1, wt=wt, _fold=C, bnf_mask=bnf_mask, _g22=g)
        if bnf is not None:
            return r[0].view(B, 2, 2, C), r[1]
        return r.view(B, 2, 2, C)
    B, H, W, C = in_shape
    K = dy.shape[3] if _g22 else w.shape[0]
    sh, sw = stride
    ph, pw = pad
    OH, OW = out_hw(H, W, KH, KW, sh, sw, ph, pw)
    if tuple(dy.shape) != (B, OH, OW, K):
        raise ValueError(f"dy shape {tuple(dy.shape)} != {(B, OH, OW, K)}")
    if _g22:
        if (KH, KW) != (1, 1) or not _g22_weight_ok(w, K, C):
            raise ValueError(f"gathered unrolled weight {tuple(w.shape)} does not match the 1x1 form {K}x{C}")
    elif tuple(w.shape) != (K, KH, KW, C):
        raise ValueError(f"weight shape {tuple(w.shape)} != {(K, KH, KW, C)}")
    if K % 8 or C % 8:
        raise ValueError("channels must be multiples of 8")
    if out is None:
        out = torch.empty((B, H, W, C), dtype=BF16, device=dy.device)
    if addend is not None:
        _chk(addend, BF16, "addend")
        assert addend.shape == out.shape
    r0, r1, s0, s1 = tap_window(H, W, KH, KW, sh, sw, ph, pw)
    M = B * H * W
    ntap = (r1 - r0) * (s1 - s0)
    hp = None if (cfg is not None or _g22) else halo_dgrad_plan(C, K, H, W, KH, KW, stride, pad)
    bm, bn, bk, splits, variant = _norm_cfg(cfg or hp or plan_conv("dgrad", M, C, ntap * K))
    if variant == HALO and (_g22 or not halo_dgrad_ok(C, K, H, W, KH, KW, stride, pad, bm, bn)):
        bm, bn, bk, splits, variant = _norm_cfg(plan_conv("dgrad", M, C, ntap * K))
    gather = not gemm1x1_ok(C, K, H, W, KH, KW, stride, pad)   # implicit GEMM: A gathered from dy per K-tile
    if variant == GEMM1X1 and ((bm, bn, bk) not in _GEMM1X1_TILES or bk > 4 or _fold or _g22 or wt is not None or
                               (gather and not gemm_dgrad_gather_ok(C, K, stride)) or not dy.is_contiguous() or
                               not out.is_contiguous()):
        bm, bn, bk, splits, variant = _GEMM1X1_FALLBACK[bm] if bm in _GEMM1X1_FALLBACK else \
            _norm_cfg(default_plan("dgrad", M, C, ntap * K))
    plan = (bm, bn, bk, splits, variant)
    if variant == GEMM1X1:  # dx[M, C] = dy[M, K] @ w[K, C] on the MFMA GEMM, the dgrad epilogue fused
        by, bc, bmean, brstd, part, rows, grp, gcnt, tpg, G = _bnf_ws(bnf, out, M, C, plan)
        from . import gemm as GM
        if gather:
            HIP.call("kml_gemm_conv_dgrad", "p p p p p p p p p i p i i i i i i i i i i p p i s", _p(dy), _p(w),
                     _p(out), _p(addend), _p(by), _p(bc), _p(bmean), _p(brstd), _p(rows),
                     int(bool(bnf_mask) and bnf is not None), _p(GM._zp(dy.device)), B, H, W, C, K, KH, KW, ph, pw,
                     bk, _p(grp), _p(gcnt), tpg, _s())
            return (out, (part, G)) if bnf is not None else out
        HIP.call("kml_gemm_dgrad_bnf", "p l p l p l p p p p p p i p i i i i p p i s", _p(dy), K, _p(w), C, _p(out), C,
                 _p(addend), _p(by), _p(bc), _p(bmean), _p(brstd), _p(rows),
                 int(bool(bnf_mask) and bnf is not None), _p(GM._zp(dy.device)), M, C, K, bk, _p(grp), _p(gcnt), tpg,
                 _s())
        return (out, (part, G)) if bnf is not None else out
    if s2_parity_ok(B, H, W, stride, plan, _g22, _fold, operands=addend is not None or bnf is not None):
        part, G = None, 0
        by = bc = bmean = brstd = None
        if bnf is not None:
            by, bc, bmean, brstd = bnf
            if bc.shape != out.shape or (by is not None and by.shape != out.shape):
                raise ValueError("bnf tensors must match the dgrad output shape")
            G = HIP.fn("kml_conv_dgrad_s2_rows", "i i i i")(B, H, W, bm)
            part = torch.empty(G * 2 * C, dtype=F32, device=out.device)
        HIP.call("kml_conv_dgrad_s2", "p p p p p p p p p i i i i i i i i i i i i i i s",
                 _p(dy), _p(w), _p(out), _p(addend), _p(by), _p(bc), _p(bmean), _p(brstd), _p(part), B, H, W, C, K,
                 KH, KW, ph, pw, bm, bn, bk, variant, int(bool(bnf_mask) and bnf is not None), _s())
        return (out, (part, G)) if bnf is not None else out
    by, bc, bmean, brstd, part, rows, grp, gcnt, tpg, G = _bnf_ws(bnf, out, M, C, plan, _fold)
    slab = cnt = None
    if variant in (HALO, ONESHOT):
        wt, splits, bk = None, 1, 0
    elif variant == DIRECT:
        if _g22:
            raise ValueError("the direct dgrad variant needs a materialised unrolled weight (not GATHER22)")
        # k-contiguous transposed weight copy, then the LDS-free kernel (bk = wave count)
        wt = _direct_wt(w, wt)
        splits = 1
    else:
        wt = None
        splits = effective_splits(ntap * _cdiv(K, bk) * bk, bk, splits)
        slab, cnt = _splitk_ws(dy.device, M, C, bm, bn, splits)
    HIP.call("kml_conv_dgrad", "p p p p p p p p p p p p i i i i i i i i i i i i i i i i i p p i i i s",
             _p(dy), _p(w), _p(wt), _p(out), _p(addend), _p(by), _p(bc), _p(bmean), _p(brstd), _p(rows), _p(grp),
             _p(gcnt), tpg, B, H, W, C, K, KH, KW, sh, sw, ph, pw, bm, bn, bk, splits, variant, _p(slab), _p(cnt),
             int(_fold), int(bool(bnf_mask) and bnf is not None), int(_g22), _s())
    return (out, (part, G)) if bnf is not None else out


# Stride-2 dgrads of the large-map convs run as four parity-class launches
# (kml_conv_dgrad_s2): 1/4 of the (pixel, tap) pairs of a stride-2 dgrad are non-zero.  Off
# for small maps (ResNet-34/CIFAR), where four launches cost more than the skipped zeros.
_S2_PARITY_MIN_ROWS = 20000


_S2_OK: dict = {}


# 1x1 / stride-1 / pad-0 conv weight gradients are plain GEMMs (dw[K][C] = dy^T x over the
# pixels).  ``wgrad_gemm.json`` maps (pixels, K, C) to the GEMM that measured faster than the
# implicit-GEMM wgrad inside the step (tools/wgrad_1x1.py): ["slab", BM, BN, stages, splits]
# (gemm.hip's deterministic slab split-K) or ["gather", ...] (the implicit GEMM on the GEMM tiles).
_WGRAD_GEMM_FILE = os.environ.get("KUBEML_WGRAD_GEMM_FILE") or \
    os.path.join(os.path.dirname(os.path.abspath(__file__)), "wgrad_gemm.json")
_WGRAD_GEMM: dict = {}
if os.path.exists(_WGRAD_GEMM_FILE):
    with open(_WGRAD_GEMM_FILE) as _f:
        for _e in json.load(_f).get("entries", []):
            # key: (input pixels, K, C, KH, stride); 1x1/s1 entries omit KH / S
            _WGRAD_GEMM[(int(_e["P"]), int(_e["K"]), int(_e["C"]), int(_e.get("KH", 1)), int(_e.get("S", 1)))] = \
                tuple(_e["route"])


def wgrad_gemm_route(x_shape, K, KH, KW, stride, pad, dbias=None):
    """The table's GEMM route for this conv's weight gradient, or None (implicit-GEMM wgrad):
    ["slab", ...] for 1x1/s1 convs (a plain GEMM), ["gather", BM, BN, stages, splits] for
    the implicit GEMM on the GEMM tiles (kml_gemm_conv_wgrad: square kernel, pad (KH - 1) / 2)."""
    if not _WGRAD_GEMM or dbias is not None or KH != KW or stride[0] != stride[1]:
        return None
    B, H, W, C = x_shape
    r = _WGRAD_GEMM.get((B * H * W, K, C, KH, stride[0]))
    if r is None:
        return None
    if r[0] == "gather":
        ok = tuple(pad) == ((KH - 1) // 2,) * 2 and C % 8 == 0 and K % 4 == 0
    elif r[0] != "slab":
        raise ValueError(f"wgrad_gemm.json: unknown route {r!r} (slab / gather: hand-written GEMMs only)")
    else:
        ok = (KH, KW) == (1, 1) and tuple(stride) == (1, 1) and tuple(pad) == (0, 0)
    return r if ok else None


def _wgrad_gemm(route, x, dy, dw, accumulate, stride=(1, 1)):
    B, H, W, C = x.shape
    K, P = dy.shape[3], B * H * W
    if route[0] == "gather":
        from . import gemm as G
        _, bm, bn, st, splits = route
        KH = dw.shape[1]
        pad = (KH - 1) // 2
        OH, OW = dy.shape[1], dy.shape[2]
        sh = int(stride[0])
        Pout = B * OH * OW
        chunk = _cdiv(_cdiv(Pout, max(1, splits)), 64) * 64
        nz = _cdiv(Pout, chunk)
        N = dw.numel() // K
        slab = torch.empty(nz * K * N, dtype=F32, device=dw.device)
        tile = G.TILES[(bm, bn, st) if st else (bm, bn)]
        HIP.call("kml_gemm_conv_wgrad", "p p p p p i i i i i i i i i i i f i i s", _p(x), _p(dy), _p(dw), _p(slab),
                 _p(G._zp(x.device)), B, H, W, C, K, KH, KH, sh, sh, pad, pad, 1.0 if accumulate else 0.0, tile,
                 int(splits), _s())
        return dw
    x2, dy2, dw2 = x.reshape(P, C), dy.reshape(P, K), dw.view(K, C)
    from . import gemm as G
    _, bm, bn, st, splits = route
    G.wgrad_splitk_(dw2, dy2, K, x2, C, K, C, P, beta=1.0 if accumulate else 0.0,
                    tile=(bm, bn, st) if st else (bm, bn), splits=splits)
    return dw


def s2_parity_ok(B, H, W, stride, plan, g22=False, fold=0, operands=True) -> bool:
    """True when a stride-2 dgrad runs as parity classes: large map, a plain igemm / glds plan
    whose tile takes the row-pass epilogue, and an addend or consumer-BN operand."""
    bm, bn, bk, _, variant = plan
    if not (tuple(stride) == (2, 2) and variant in (0, 1, 2) and not g22 and not fold and operands
            and B * H * W >= _S2_PARITY_MIN_ROWS):
        return False
    key = (bm, bn, bk, variant)
    ok = _S2_OK.get(key)
    if ok is None:
        ok = _S2_OK[key] = bool(HIP.fn("kml_conv_dgrad_s2_ok", "i i i i")(bm, bn, bk, variant))
    return ok


def _bnf_ws(bnf, out, M, C, plan, fold=0):
    """Consumer-BN partial-row buffers of a dgrad: (y, c, mean, rstd, part the BN reads,
    rows the epilogue writes, group output, tickets, tiles per group, rows in part).
    fold: the BN's channel count when the dgrad output holds C / fold positions per row."""
    if bnf is None:
        return None, None, None, None, None, None, None, None, 0, 0
    by, bc, bmean, brstd = bnf
    if bc.shape != out.shape or (by is not None and by.shape != out.shape):
        raise ValueError("bnf tensors must match the dgrad output shape")
    G = conv_stats_rows(M, plan)
    part = torch.empty(G * 2 * C, dtype=F32, device=out.device)
    rows, grp, gcnt, tpg = _stats_ws(out.device, M, C, plan, part)
    if fold:
        if grp is not None or C % fold:
            raise ValueError("folded BN partials cannot be group-reduced")
        G *= C // fold
    return by, bc, bmean, brstd, part, rows, grp, gcnt, tpg, G


def _direct_wt(w, wt):
    """Transposed weights [Cin][KH][KW][Kp] for the direct dgrad (made here when not given)."""
    K, KH, KW, C = w.shape
    Kp = _cdiv(K, 32) * 32
    if wt is None:
        wt = torch.empty((C, KH, KW, Kp), dtype=BF16, device=w.device)
        HIP.call("kml_weight_transpose", "p p i i i i s", _p(w), _p(wt), K, KH, KW, C, _s())
    elif tuple(wt.shape) != (C, KH, KW, Kp) or wt.dtype != BF16:
        raise ValueError("transposed weight shape mismatch")
    return wt


def dgrad_plan(in_shape, K, KH, KW, stride, pad, cfg=None):
    """The (bm, bn, bk, splits, variant) plan conv_dgrad runs for this conv."""
    B, H, W, C = in_shape
    r0, r1, s0, s1 = tap_window(H, W, KH, KW, stride[0], stride[1], pad[0], pad[1])
    return _norm_cfg(cfg or plan_conv("dgrad", B * H * W, C, (r1 - r0) * (s1 - s0) * K))


def bwd_plans(in_shape, K, KH, KW, stride, pad, dcfg=None, wcfg=None, unroll=False):
    """(dgrad plan, wgrad plan, grouped?) conv_bwd runs for this conv: a tuned pair entry
    when one exists, else the separately tuned plans (grouped if instantiated).
    unroll: plans of the unrolled 1x1 form (:func:`unrolled22`)."""
    B, H, W, C = in_shape
    if unroll:
        return bwd_plans((B, 1, 1, 4 * C), 4 * K, 1, 1, (1, 1), (0, 0), dcfg, wcfg)
    sh, sw = stride
    ph, pw = pad
    OH, OW = out_hw(H, W, KH, KW, sh, sw, ph, pw)
    r0, r1, s0, s1 = tap_window(H, W, KH, KW, sh, sw, ph, pw)
    ntap = (r1 - r0) * (s1 - s0)
    if dcfg is None and wcfg is None:
        dcfg, wcfg = _TUNED_PAIR.get((B * H * W, C, ntap * K, K, ntap * C, B * OH * OW), (None, None))
        hp = halo_dgrad_plan(C, K, H, W, KH, KW, stride, pad)
        if hp is not None:
            dcfg = hp
        od, ow = oneshot_bwd_plans(C, K, B, H, W, KH, KW, stride, pad)
        dcfg, wcfg = od or dcfg, ow or wcfg
    dplan = _norm_cfg(dcfg or plan_conv("dgrad", B * H * W, C, ntap * K))
    wplan = _norm_cfg(wcfg or plan_conv("wgrad", K, ntap * C, B * OH * OW))
    return dplan, wplan, conv_pair_supported(dplan, wplan)


_PAIR_OK: dict = {}


def conv_pair_supported(dcfg, wcfg) -> bool:
    """True if the (dgrad plan, wgrad plan) combination has a grouped one-launch kernel."""
    key = (tuple(dcfg), tuple(wcfg))
    ok = _PAIR_OK.get(key)
    if ok is None:
        dbm, dbn, dbk, _, dv = dcfg
        wbm, wbn, wbk, _, wv = wcfg
        ok = _PAIR_OK[key] = bool(HIP.fn("kml_conv_pair_supported", "i i i i i i i i")(
            dv, dbm, dbn, dbk, wv, wbm, wbn, wbk))
    return ok


def conv_bwd(dy, w, x, dw, KH, KW, stride, pad, addend=None, bnf=None, wt=None, dcfg=None, wcfg=None, wu=None,
             bnf_mask=False, accumulate=True, dbias=None, bias_accumulate=True, rider=None):
    """Both backward GEMMs of a conv: dx (+addend, + consumer-BN partials as in
    :func:`conv_dgrad`) and ``dw += wgrad`` (``accumulate=False``: ``dw = wgrad``).  Runs as ONE grouped launch
    (``k_conv_pair``: dgrad tiles and wgrad tiles share a grid) when the two plans have an
    instantiated pair, else as two launches.  ``wt``: precomputed transposed weights for
    a direct-variant dgrad (:func:`weight_transpose_multi`); made here when missing.
    Returns dx, or (dx, (part, G)) when ``bnf`` is given.  wu: unrolled weight
    (:func:`unrolled22`): both GEMMs run in the dense 1x1 form; ``dw`` is then the
    ``[4K,1,1,4C]`` fp32 scratch of the 1x1-form weight gradient (stored), which
    :func:`fold22_multi` folds onto the 3x3 taps.  bnf_mask: as in :func:`conv_dgrad`.
    dbias: as in :func:`conv_wgrad` (1x1/s1/p0 convs).
    rider: an :class:`SgdRider` applied by extra blocks of the grouped launch (or by its own
    launch after the two GEMMs when this conv does not run grouped)."""
    _chk(dy, BF16, "dy", 4)
    _chk(w, BF16, "w", 4)
    _chk(x, BF16, "x", 4)
    _chk(dw, F32, "dw", 4)
    B, H, W, C = x.shape
    K = w.shape[0]
    sh, sw = stride
    ph, pw = pad
    OH, OW = out_hw(H, W, KH, KW, sh, sw, ph, pw)
    want_dw = (4 * K, 1, 1, 4 * C) if wu is not None else (K, KH, KW, C)
    if tuple(dy.shape) != (B, OH, OW, K) or tuple(w.shape) != (K, KH, KW, C) or tuple(dw.shape) != want_dw:
        raise ValueError("conv_bwd shape mismatch")
    if K % 8 or C % 8:
        raise ValueError("channels must be multiples of 8")
    fold, g22 = 0, False
    if wu is not None:
        _check_wu(x.shape, w, wu, KH, KW, stride, pad)
        dy, x, addend, bnf = _u22_views(B, C, K, dy=dy, x=x, addend=addend, bnf=bnf)
        g22 = wu is GATHER22
        w, fold, accumulate = (w if g22 else wu), C, False
        H = W = OH = OW = 1
        KH = KW = sh = sw = 1
        ph = pw = 0
        C, K = 4 * C, 4 * K
        stride, pad = (1, 1), (0, 0)
    r0, r1, s0, s1 = tap_window(H, W, KH, KW, sh, sw, ph, pw)
    ntap = (r1 - r0) * (s1 - s0)
    M = B * H * W
    dplan, wplan, grouped = bwd_plans(x.shape, K, KH, KW, stride, pad, dcfg, wcfg)
    wroute = None if (wcfg is not None or wu is not None) else wgrad_gemm_route(x.shape, K, KH, KW, stride, pad, dbias)
    if wroute is not None:
        grouped = False
    if grouped and s2_parity_ok(B, H, W, stride, dplan, g22, fold, operands=addend is not None or bnf is not None):
        grouped = False
    if dbias is not None and wu is not None:
        raise ValueError("conv_bwd: dbias needs a 1x1 conv")
    if not grouped:
        conv_wgrad(x, dy, dw, KH, KW, stride, pad, cfg=None if wroute is not None else wplan, accumulate=accumulate,
                   dbias=dbias, bias_accumulate=bias_accumulate)
        r = conv_dgrad(dy, w, (B, H, W, C), KH, KW, stride, pad, addend=addend, cfg=dplan, bnf=bnf, wt=wt, _fold=fold,
                       bnf_mask=bnf_mask, _g22=g22)
        if rider is not None:
            rider.run_alone()
        if not fold:
            return r
        if bnf is not None:
            return r[0].view(B, 2, 2, C // 4), r[1]
        return r.view(B, 2, 2, C // 4)
    bm, bn, bk, splits, variant = dplan
    out = torch.empty((B, H, W, C), dtype=BF16, device=dy.device)
    if addend is not None:
        _chk(addend, BF16, "addend")
        assert addend.shape == out.shape
    by, bc, bmean, brstd, part, rows, grp, gcnt, tpg, G = _bnf_ws(bnf, out, M, C, dplan, fold)
    slab = cnt = None
    if variant in (HALO, ONESHOT):
        wt, dsplits = None, 1
    elif variant == DIRECT:
        if g22:
            raise ValueError("the direct dgrad variant needs a materialised unrolled weight (not GATHER22)")
        wt = _direct_wt(w, wt)
        dsplits = 1
    else:
        wt = None
        dsplits = effective_splits(ntap * _cdiv(K, bk) * bk, bk, splits)
        slab, cnt = _splitk_ws(dy.device, M, C, bm, bn, dsplits)
    wbm, wbn, wbk, wsplits, wvariant = wplan
    _chk_dbias(dbias, K, KH, KW, stride, pad)
    wslab, wcnt = _wgrad_ws(dw.device, B, H, W, C, K, KH, KW, stride, pad, wplan, dbias is not None)
    with _Riding(rider):
        HIP.call("kml_conv_bwd_pair",
                 "p p p p p p p p p p p p i p p i i i i i i i i i i i i i i i i p p i i i i i i i p p i p i i s",
                 _p(dy), _p(w), _p(wt), _p(out), _p(addend), _p(by), _p(bc), _p(bmean), _p(brstd), _p(rows),
                 _p(grp), _p(gcnt), tpg, _p(x), _p(dw), B, H, W, C, K, KH, KW, sh, sw, ph, pw, bm, bn, bk, dsplits,
                 variant, _p(slab), _p(cnt), wbm, wbn, wbk, wsplits, wvariant, int(fold),
                 int(bool(bnf_mask) and bnf is not None), _p(wslab), _p(wcnt), int(bool(accumulate)), _p(dbias),
                 int(bool(bias_accumulate)), int(g22), _s())
    if fold:
        out = out.view(B, 2, 2, C // 4)
    return (out, (part, G)) if bnf is not None else out


def weight_transpose_multi(ws, wts):
    """wts[i][C,KH,KW,Kp] = transpose of ws[i][K,KH,KW,C] (Kp = roundup(K, 32), zero pad) for
    up to 16 weights in one launch (direct-variant dgrad operands)."""
    import ctypes
    n = len(ws)
    if n == 0:
        return
    if n > 16 or len(wts) != n:
        raise ValueError("weight_transpose_multi: 1..16 pairs")
    wp = (ctypes.c_void_p * n)()
    tp = (ctypes.c_void_p * n)()
    dims = (ctypes.c_int * (4 * n))()
    for i, (w, wt) in enumerate(zip(ws, wts)):
        _chk(w, BF16, "w", 4)
        _chk(wt, BF16, "wt", 4)
        K, KH, KW, C = w.shape
        if tuple(wt.shape) != (C, KH, KW, _cdiv(K, 32) * 32):
            raise ValueError("transposed weight shape mismatch")
        wp[i], tp[i] = w.data_ptr(), wt.data_ptr()
        dims[4 * i], dims[4 * i + 1], dims[4 * i + 2] = K, KH * KW, C
    HIP.call("kml_weight_transpose_multi", "p p p i s", ctypes.addressof(wp), ctypes.addressof(tp),
             ctypes.addressof(dims), n, _s())


def _wgrad_ws(device, B, H, W, C, K, KH, KW, stride, pad, cfg, bias_col=False):
    """Split-K slab + tickets of a weight-gradient GEMM (None, None without split-K);
    bias_col: the GEMM carries the extra ones column of a fused bias gradient."""
    bm, bn, bk, splits, variant = cfg
    if variant:
        bk = 64
    OH, OW = out_hw(H, W, KH, KW, stride[0], stride[1], pad[0], pad[1])
    r0, r1, s0, s1 = tap_window(H, W, KH, KW, stride[0], stride[1], pad[0], pad[1])
    return _splitk_ws(device, K, (r1 - r0) * (s1 - s0) * C + int(bias_col), bm, bn,
                      effective_splits(B * OH * OW, bk, splits))


def _chk_dbias(dbias, K, KH, KW, stride, pad):
    if dbias is None:
        return
    _chk(dbias, F32, "dbias")
    if dbias.numel() < K or (KH, KW) != (1, 1) or tuple(stride) != (1, 1) or tuple(pad) != (0, 0):
        raise ValueError("fused bias gradient: 1x1/s1/p0 conv and a [Cout] fp32 dbias")


def conv_wgrad(x, dy, dw, KH, KW, stride, pad, cfg=None, unroll=False, accumulate=True, dbias=None,
               bias_accumulate=True, rider=None):
    """Conv weight gradient into dw[Cout,KH,KW,Cin] (fp32): ``dw += wgrad`` (accumulate) or
    ``dw = wgrad`` (overwrite: the buffer need not be zeroed).  Deterministic: one writer per
    element, split-K partials summed in split order.  unroll: an unrolled conv
    (:func:`unrolled22`): ``dw`` is then the ``[4K,1,1,4C]`` fp32 scratch of its dense 1x1-form
    gradient, stored; :func:`fold22_multi` folds it onto the 3x3 taps.  dbias (1x1/s1/p0 convs,
    i.e. a Linear): the bias gradient sum over pixels of dy, from the same GEMM (an extra
    ones column of the input operand), stored or added per ``bias_accumulate``."""
    _chk(x, BF16, "x", 4)
    _chk(dy, BF16, "dy", 4)
    _chk(dw, F32, "dw", 4)
    if unroll:
        if dbias is not None:
            raise ValueError("conv_wgrad: dbias needs a 1x1 conv")
        B, H, W, C = x.shape
        K = dy.shape[3]
        if not unrolled22(H, W, KH, KW, stride, pad) or tuple(dw.shape) != (4 * K, 1, 1, 4 * C):
            raise ValueError("unrolled wgrad: needs the [4K,1,1,4C] fp32 scratch")
        _, x1, _, _ = _u22_views(B, C, K, x=x)
        return conv_wgrad(x1, dy.reshape(B, 1, 1, 4 * K), dw, 1, 1, (1, 1), (0, 0), cfg=cfg, accumulate=False,
                          rider=rider)
    B, H, W, C = x.shape
    K = dy.shape[3]
    sh, sw = stride
    ph, pw = pad
    OH, OW = out_hw(H, W, KH, KW, sh, sw, ph, pw)
    if tuple(dy.shape) != (B, OH, OW, K) or tuple(dw.shape) != (K, KH, KW, C):
        raise ValueError("wgrad shape mismatch")
    route = None if cfg is not None else wgrad_gemm_route(x.shape, K, KH, KW, stride, pad, dbias)
    if route is not None:
        r = _wgrad_gemm(route, x, dy, dw, accumulate, stride)
        if rider is not None:
            rider.run_alone()
        return r
    r0, r1, s0, s1 = tap_window(H, W, KH, KW, sh, sw, ph, pw)
    cfg = _norm_cfg(cfg or plan_conv("wgrad", K, (r1 - r0) * (s1 - s0) * C, B * OH * OW))
    bm, bn, bk, splits, variant = cfg
    _chk_dbias(dbias, K, KH, KW, stride, pad)
    slab, cnt = _wgrad_ws(dw.device, B, H, W, C, K, KH, KW, stride, pad, cfg, dbias is not None)
    with _Riding(rider):   # the register-staged wgrad carries it in extra z-slices (else its own launch)
        HIP.call("kml_conv_wgrad", "p p p i i i i i i i i i i i i i i i i i p p p i s",
                 _p(x), _p(dy), _p(dw), B, H, W, C, K, KH, KW, sh, sw, ph, pw, bm, bn, bk, splits, variant,
                 int(bool(accumulate)), _p(slab), _p(cnt), _p(dbias), int(bool(bias_accumulate)), _s())
    return dw


def fold22_multi(jobs):
    """jobs: [(g [4K,1,1,4C] fp32, dw [K,3,3,C] fp32 region, accumulate)] — the unrolled convs'
    weight gradients folded onto their 3x3 taps (fixed pair order, no atomics), 16 per launch."""
    import ctypes
    for i in range(0, len(jobs), 16):
        part = jobs[i:i + 16]
        n = len(part)
        gp = (ctypes.c_void_p * n)()
        dp = (ctypes.c_void_p * n)()
        dims = (ctypes.c_int * (3 * n))()
        for k, (g, dw, acc) in enumerate(part):
            _chk(g, F32, "g", 4)
            _chk(dw, F32, "dw", 4)
            K, _, _, C = dw.shape
            if tuple(dw.shape) != (K, 3, 3, C) or tuple(g.shape) != (4 * K, 1, 1, 4 * C):
                raise ValueError("fold22_multi: shape mismatch")
            gp[k], dp[k] = g.data_ptr(), dw.data_ptr()
            dims[3 * k], dims[3 * k + 1], dims[3 * k + 2] = K, C, int(bool(acc))
        HIP.call("kml_conv_fold22_multi", "p p p i s", ctypes.addressof(gp), ctypes.addressof(dp),
                 ctypes.addressof(dims), n, _s())


# --------------------------------------------------------------------------------------
# batch norm / relu / elementwise
# --------------------------------------------------------------------------------------

def bn_stats(x2d, stats):
    """stats[2C] += [sum, sumsq] (atomics)."""
    _chk(x2d, BF16, "x")
    M, C = x2d.numel() // x2d.shape[-1], x2d.shape[-1]
    HIP.call("kml_bn_stats", "p p l i s", _p(x2d), _p(stats), M, C, _s())


def bn_stats_part(x2d):
    """Per-block partial [sum | sumsq] rows -> (buffer [G*2C], G) for bn_apply(stats_rows=G)."""
    _chk(x2d, BF16, "x")
    M, C = x2d.numel() // x2d.shape[-1], x2d.shape[-1]
    G = HIP.raw("kml_bn_stats_rows", M, C)
    part = torch.empty(G * 2 * C, dtype=F32, device=x2d.device)
    HIP.call("kml_bn_stats_part", "p p l i s", _p(x2d), _p(part), M, C, _s())
    return part, G


def _fold_ws(G, C, dev):
    """Workspace for folding a large [G][2C] partial-row buffer (kml_bn_fold_rows) or None."""
    n = HIP.fn("kml_bn_fold_rows", "i i")(int(G), int(C))
    return torch.empty(n * 2 * C, dtype=F32, device=dev) if n > 0 else None


def bn_apply(x, stats, gamma, beta, y=None, res=None, save_mean=None, save_rstd=None, run_mean=None,
             run_var=None, eps=1e-5, momentum=0.1, relu=False, training=True, stats_rows=0):
    _chk(x, BF16, "x")
    C = x.shape[-1]
    M = x.numel() // C
    if y is None:
        y = torch.empty_like(x)
    if res is not None:
        _chk(res, BF16, "res")
        if res.shape != x.shape:
            raise ValueError("residual shape mismatch")
    ws = _fold_ws(stats_rows, C, x.device) if training and stats_rows > 0 else None
    args = (_p(x), _p(stats), int(stats_rows), _p(gamma), _p(beta), _p(res), _p(y), _p(save_mean), _p(save_rstd),
            _p(run_mean), _p(run_var), M, C, float(eps), float(momentum), int(relu), 0 if training else 1, _p(ws))
    if _BN_PAIR is not None and len(_BN_PAIR) < 2:   # the record holds every operand until the launch
        _BN_PAIR.append((args, (x, stats, gamma, beta, res, y, save_mean, save_rstd, run_mean, run_var, ws)))
        return y
    HIP.call("kml_bn_apply", _BN_SIG, *args, _s())
    return y


_BN_SIG = "p p i p p p p p p p p l i f f i i p s"
_BN_PAIR = None   # list while a bn_apply_pair() block records
BN_PAIRS_LAUNCHED = [0]


@contextlib.contextmanager
def bn_apply_pair():
    """Launch the (up to) two bn_apply calls made inside this block as ONE kernel (bn.hip
    k_bn_apply_pair) when both take the single-batch register path; otherwise each launches on its
    own at the end of the block.  The applies must not depend on each other."""
    global _BN_PAIR
    prev, _BN_PAIR = _BN_PAIR, []
    try:
        yield
    finally:
        rec, _BN_PAIR = _BN_PAIR, prev
        rc = 1
        if len(rec) == 2:
            import ctypes
            import struct

            def q(a):
                v = [int(t) if not isinstance(t, float) else struct.unpack("<I", struct.pack("<f", t))[0] for t in a]
                return (ctypes.c_longlong * 18)(*v)
            qs = [q(a) for a, _ in rec]
            rc = HIP.fn("kml_bn_apply_pair", "p p s")(ctypes.addressof(qs[0]), ctypes.addressof(qs[1]), _s())
        if rc == 1:
            for a, _ in rec:
                HIP.call("kml_bn_apply", _BN_SIG, *a, _s())
        elif rc:
            raise RuntimeError(f"kml_bn_apply_pair failed: {rc}")
        else:
            BN_PAIRS_LAUNCHED[0] += 1


# BN-backward dgamma/dbeta reduction: "fused" (default) = per-block partials, summed in
# a fixed order by the apply kernel (deterministic, no atomics / fences); "ticket" = the
# in-kernel last-arriver reduce; "atomic" = fp32 atomics (tests and tools/bn_micro.py compare).
_BN_REDUCE = "fused"


def bn_bwd(dy, y, x, mean, rstd, gamma, dgamma, dbeta, dx=None, dres=None, partial=None, accumulate=True,
           rider=None):
    """dgamma/dbeta (``+=``, or ``=`` with accumulate=False) and dx; y given => ReLU mask
    applied; dres (optional) receives dz.  partial = (part, G) from conv_dgrad(bnf=...) skips
    the reduction pass.  rider: an :class:`SgdRider` run by extra blocks of the apply launch."""
    _chk(dy, BF16, "dy")
    _chk(x, BF16, "x")
    C = x.shape[-1]
    M = x.numel() // C
    if dx is None:
        dx = torch.empty_like(x)
    record = _BNB_PAIR is not None and len(_BNB_PAIR) < 2 and rider is None
    if partial is not None:
        part, G = partial
        fws = _fold_ws(G, C, dy.device)
        args = (_p(dy), _p(y), _p(x), _p(mean), _p(rstd), _p(gamma), _p(part), int(G), _p(dgamma), _p(dbeta),
                _p(dx), _p(dres), M, C, _p(fws), int(bool(accumulate)))
        if record:
            _BNB_PAIR.append(((1,) + args, (dy, y, x, mean, rstd, gamma, part, dgamma, dbeta, dx, dres, fws)))
            return dx
        with _Riding(rider):
            HIP.call("kml_bn_bwd_apply_partial", "p p p p p p p i p p p p l i p i s", *args, _s())
        return dx
    ws = cnt = None
    if _BN_REDUCE in ("fused", "ticket"):
        nws = HIP.raw("kml_bn_bwd_ws_floats", M, C)
        ws = torch.empty(nws, dtype=F32, device=x.device)
        if _BN_REDUCE == "ticket":
            cnt = _COUNTERS.take(x.device, 1)
    args = (_p(dy), _p(y), _p(x), _p(mean), _p(rstd), _p(gamma), _p(dgamma), _p(dbeta), _p(dx), _p(dres), _p(ws),
            _p(cnt), M, C, int(bool(accumulate)))
    if record:   # the record holds every operand (the reduction workspace included) until the launch
        _BNB_PAIR.append(((0,) + args, (dy, y, x, mean, rstd, gamma, dgamma, dbeta, dx, dres, ws, cnt)))
        return dx
    with _Riding(rider):
        HIP.call("kml_bn_bwd", "p p p p p p p p p p p p l i i s", *args, _s())
    return dx


_BNB_PAIR = None   # list while a bn_bwd_pair() block records
BNB_PAIRS = [0]    # bn_bwd_pair() blocks that recorded two calls (tests)


@contextlib.contextmanager
def bn_bwd_pair():
    """Run the (up to) two bn_bwd calls made inside this block at its end with ONE apply launch
    (bn.hip kml_bn_bwd_pair / k_bn_bwd_apply_pair) when both applies take the single-batch
    register path; their reduction passes, if any, run first.  A call with a rider launches at
    once, as always.  The two BN backwards must not depend on each other."""
    global _BNB_PAIR
    import ctypes
    prev, _BNB_PAIR = _BNB_PAIR, []
    try:
        yield
    finally:
        rec, _BNB_PAIR = _BNB_PAIR, prev
        if len(rec) == 2:
            qs = [(ctypes.c_longlong * 17)(*[int(v) for v in a]) for a, _ in rec]
            HIP.call("kml_bn_bwd_pair", "p p s", ctypes.addressof(qs[0]), ctypes.addressof(qs[1]), _s())
            BNB_PAIRS[0] += 1
        else:
            for a, _ in rec:
                if a[0] == 1:
                    HIP.call("kml_bn_bwd_apply_partial", "p p p p p p p i p p p p l i p i s", *a[1:], _s())
                else:
                    HIP.call("kml_bn_bwd", "p p p p p p p p p p p p l i i s", *a[1:], _s())


def relu_fwd(x):
    y = torch.empty_like(x)
    HIP.call("kml_relu_fwd", "p p l s", _p(x), _p(y), x.numel(), _s())
    return y


def relu_bwd(dy, y):
    dx = torch.empty_like(dy)
    HIP.call("kml_relu_bwd", "p p p l s", _p(dy), _p(y), _p(dx), dy.numel(), _s())
    return dx


def add_bf16(a, b, out=None):
    out = torch.empty_like(a) if out is None else out
    HIP.call("kml_add_bf16", "p p p l s", _p(a), _p(b), _p(out), a.numel(), _s())
    return out


def fill_(t, value=0.0):
    """fp32 fill with a kernel (graph-safe alternative to a memset node)."""
    _chk(t, F32, "t")
    HIP.call("kml_fill_f32", "p f l s", _p(t), float(value), t.numel(), _s())
    return t


_ZR_MAX = None


def zero_ranges_max() -> int:
    global _ZR_MAX
    if _ZR_MAX is None:
        _ZR_MAX = int(HIP.raw("kml_zero_ranges_max"))
    return _ZR_MAX


def zero_ranges_(t, runs):
    """Zero [offset, offset + n) element runs of the fp32 buffer ``t`` in one launch
    (offsets multiples of 4; at most :func:`zero_ranges_max` runs)."""
    import ctypes
    _chk(t, F32, "t")
    k = len(runs)
    if k == 0:
        return t
    if k > zero_ranges_max():
        raise ValueError("zero_ranges_: too many runs")
    offs = (ctypes.c_longlong * k)(*[int(o) for o, _ in runs])
    ns = (ctypes.c_int * k)(*[int(n) for _, n in runs])
    if any(int(o) + int(n) > t.numel() for o, n in runs):
        raise ValueError("zero_ranges_: run outside the buffer")
    HIP.call("kml_zero_ranges", "p p p i s", _p(t), ctypes.addressof(offs), ctypes.addressof(ns), k, _s())
    return t


def memset_(t, value=0):
    """Zero a tensor with a kernel (graph-safe; see kml_zero in util.hip)."""
    if value != 0:
        raise ValueError("only zero fill is supported")
    if not t.is_contiguous():
        raise ValueError("memset_ needs a contiguous tensor")
    HIP.call("kml_zero", "p l s", _p(t), t.numel() * t.element_size(), _s())
    return t


def f32_to_bf16(x, out=None):
    out = torch.empty(x.shape, dtype=BF16, device=x.device) if out is None else out
    HIP.call("kml_f32_to_bf16", "p p l s", _p(x), _p(out), x.numel(), _s())
    return out


def bf16_to_f32(x, out=None):
    out = torch.empty(x.shape, dtype=F32, device=x.device) if out is None else out
    HIP.call("kml_bf16_to_f32", "p p l s", _p(x), _p(out), x.numel(), _s())
    return out


def scale_(x, a):
    HIP.call("kml_scale_f32", "p f l s", _p(x), float(a), x.numel(), _s())
    return x


# --------------------------------------------------------------------------------------
# pooling
# --------------------------------------------------------------------------------------

def maxpool_fwd(x, k, s, p):
    _chk(x, BF16, "x", 4)
    B, H, W, C = x.shape
    OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    y = torch.empty((B, OH, OW, C), dtype=BF16, device=x.device)
    idx = torch.empty((B, OH, OW, C), dtype=torch.uint8, device=x.device)
    HIP.call("kml_maxpool_fwd", "p p p i i i i i i i s", _p(x), _p(y), _p(idx), B, H, W, C, k, s, p, _s())
    return y, idx


def maxpool_bwd(dy, idx, in_shape, k, s, p, relu_out=None):
    """Gather max-pool backward.  relu_out: the pooled output of :func:`bn_relu_maxpool`;
    windows whose maximum is not > 0 pass no gradient (the ReLU mask folded in)."""
    B, H, W, C = in_shape
    if relu_out is not None and relu_out.shape != dy.shape:
        raise ValueError("relu_out must have the pooled shape")
    dx = torch.empty((B, H, W, C), dtype=BF16, device=dy.device)
    HIP.call("kml_maxpool_bwd", "p p p p i i i i i i i s", _p(dy), _p(idx), _p(relu_out), _p(dx), B, H, W, C, k, s,
             p, _s())
    return dx


def shortcut_a_fwd(x, pad):
    """Option-A shortcut (CIFAR ResNet): ``F.pad(x[:, ::2, ::2, :], (pad, pad))`` on NHWC bf16
    in one gather launch.  Needs C % 8 == 0 and pad % 8 == 0."""
    _chk(x, BF16, "x", 4)
    B, H, W, C = x.shape
    if C % 8 or pad % 8 or pad < 0:
        raise ValueError(f"shortcut_a_fwd: C={C} and pad={pad} must be multiples of 8")
    y = torch.empty((B, (H + 1) // 2, (W + 1) // 2, C + 2 * pad), dtype=BF16, device=x.device)
    HIP.call("kml_shortcut_a_fwd", "p p i i i i i s", _p(x), _p(y), B, H, W, C, int(pad), _s())
    return y


def shortcut_a_bwd(dy, in_shape, pad):
    """Backward of :func:`shortcut_a_fwd`: the un-padded channels of dy at even pixels, zeros
    elsewhere (writes every element of dx — no zero-fill pass)."""
    _chk(dy, BF16, "dy", 4)
    B, H, W, C = in_shape
    if tuple(dy.shape) != (B, (H + 1) // 2, (W + 1) // 2, C + 2 * pad):
        raise ValueError("shortcut_a_bwd: dy does not match the input shape and pad")
    dx = torch.empty((B, H, W, C), dtype=BF16, device=dy.device)
    HIP.call("kml_shortcut_a_bwd", "p p i i i i i s", _p(dy), _p(dx), B, H, W, C, int(pad), _s())
    return dx


def bn_relu_maxpool(x, stats, gamma, beta, k, s, p, save_mean=None, save_rstd=None, run_mean=None, run_var=None,
                    eps=1e-5, momentum=0.1, stats_rows=0, counters=None):
    """Training BN (batch statistics from ``stats``: [stats_rows][2C] conv-epilogue partial
    rows, or final [2C] sums) -> ReLU -> max-pool(k, s, p) in one pass; returns (pooled,
    argmax idx).  The normalised map is never materialised — backward is
    ``maxpool_bwd(..., relu_out=pooled)`` then ``bn_bwd`` without a ReLU mask.  counters:
    an int64 tensor (the model's BN ``num_batches_tracked`` arena) incremented by one."""
    _chk(x, BF16, "x", 4)
    B, H, W, C = x.shape
    OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    y = torch.empty((B, OH, OW, C), dtype=BF16, device=x.device)
    idx = torch.empty((B, OH, OW, C), dtype=torch.uint8, device=x.device)
    ws = _fold_ws(stats_rows, C, x.device) if stats_rows > 0 else None
    if counters is not None and (counters.dtype != torch.int64 or not counters.is_contiguous()):
        raise ValueError("counters must be a contiguous int64 tensor")
    HIP.call("kml_bn_relu_maxpool", "p p i p p p p p p p p i i i i i i i f f p p i s",
             _p(x), _p(stats), int(stats_rows), _p(gamma), _p(beta), _p(y), _p(idx), _p(save_mean), _p(save_rstd),
             _p(run_mean), _p(run_var), B, H, W, C, k, s, p, float(eps), float(momentum), _p(ws), _p(counters),
             0 if counters is None else counters.numel(), _s())
    return y, idx


def gavgpool_fwd(x):
    B, H, W, C = x.shape
    y = torch.empty((B, C), dtype=BF16, device=x.device)
    HIP.call("kml_gavgpool_fwd", "p p i i i s", _p(x), _p(y), B, H * W, C, _s())
    return y


def gavgpool_bwd(dy, in_shape):
    B, H, W, C = in_shape
    dx = torch.empty((B, H, W, C), dtype=BF16, device=dy.device)
    HIP.call("kml_gavgpool_bwd", "p p i i i s", _p(dy), _p(dx), B, H * W, C, _s())
    return dx


# --------------------------------------------------------------------------------------
# loss
# --------------------------------------------------------------------------------------

def ce_fwd(logits, labels, ignore_index=-100, classes=None):
    """Returns (out3, ws): out3 = [mean loss, correct, valid] fp32 on device.  ``classes``:
    number of real classes when ``logits`` is [B, ld] with the rows padded past them (a
    padded Linear output used in place: no slice copy)."""
    if logits.dim() != 2:
        raise ValueError("logits must be [B, C]")
    if not logits.is_contiguous():
        logits = logits.contiguous()
    dt = {BF16: 0, F32: 1}[logits.dtype]
    B, ld = logits.shape
    C = ld if classes is None else int(classes)
    if C > ld:
        raise ValueError("classes exceeds the logits row")
    labels = labels.to(torch.int64).contiguous()
    ws = torch.empty(3 * B, dtype=F32, device=logits.device)
    out3 = torch.empty(3, dtype=F32, device=logits.device)
    ticket = _COUNTERS.take(logits.device, 1)   # in-launch fold of the per-row results
    HIP.call("kml_ce_fwd", "p p p p i i i l i p s", _p(logits), _p(labels), _p(ws), _p(out3), B, C, ld,
             int(ignore_index), dt, _p(ticket), _s())
    return out3, ws, labels


def ce_bias_fusable(logits) -> bool:
    """ce_bwd can add the logits' column sums to a bias gradient in the same pass."""
    return logits.dtype == BF16 and logits.dim() == 2 and logits.shape[1] % 8 == 0 and logits.shape[1] <= 4096


def ce_bwd(logits, labels, ws, out3, grad_out=None, ignore_index=-100, classes=None, dbias=None, accumulate=True):
    """dlogits (same [B, ld] layout as the logits; pad columns 0).  dbias (fp32, needs
    :func:`ce_bias_fusable`): the column sums of dlogits (the logits Linear's bias gradient),
    added (accumulate) or stored; deterministic (ordered partial rows, no atomics)."""
    dt = {BF16: 0, F32: 1}[logits.dtype]
    B, ld = logits.shape
    C = ld if classes is None else int(classes)
    d = torch.empty_like(logits)
    if dbias is not None:
        _chk(dbias, F32, "dbias")
        if not ce_bias_fusable(logits) or dbias.numel() < C:
            raise ValueError("ce_bwd: bias fusion needs bf16 logits with ld % 8 == 0, ld <= 4096")
    part = cnt = None
    if dbias is not None:
        part = torch.empty(_cdiv(B, 16) * _cdiv(C, 4) * 4, dtype=F32, device=logits.device)
        cnt = _COUNTERS.take(logits.device, 1)
    HIP.call("kml_ce_bwd", "p p p p p p i i i l i p p p i s", _p(logits), _p(labels), _p(ws), _p(out3), _p(grad_out),
             _p(d), B, C, ld, int(ignore_index), dt, _p(dbias), _p(part), _p(cnt), int(bool(accumulate)), _s())
    return d


# --------------------------------------------------------------------------------------
# optimizers
# --------------------------------------------------------------------------------------

def sgd_(w, g, mom, shadow, lr, wd=0.0, momentum=0.0, dampening=0.0, nesterov=False, first=False,
         grad_scale=1.0, lr_dev=None, first_dev=None, max_blocks=0, advance=None):
    """first_dev: fp32 device flag (non-zero = first step after a state reset); when given
    it overrides ``first`` so graph replays follow reset_state().  max_blocks: grid cap.
    advance: (ctr, batch, n) -- also do :func:`advance_counter_` (ctr, batch, n) in this launch."""
    n = w.numel()
    ctr, ab, an = None, 0.0, 0.0
    if advance is not None:
        ctr, ab, an = advance
        _chk(ctr, F32, "ctr")
        if ctr.numel() < 3 or ctr.device != w.device:
            raise ValueError("advance counter must be a [3] fp32 tensor on the parameters' device")
        ab, an = float(ab), float(an)
    HIP.call("kml_sgd", "p p p p p f f f f i p i f l i p f f s", _p(w), _p(g), _p(mom), _p(shadow), _p(lr_dev),
             float(lr), float(wd), float(momentum), float(dampening), int(nesterov), _p(first_dev), int(first),
             float(grad_scale), n, int(max_blocks), _p(ctr), ab, an, _s())


class SgdRider:
    """One fused-SGD range carried by a grouped conv-backward launch (``conv_bwd(rider=...)``,
    ``k_conv_pair``'s third role, csrc/include/kml_sgd.h): the same element update as
    :func:`sgd_` with the learning rate and the first-step flag read on the device, so a
    graph-captured step follows ``set_lr`` / ``reset_state``.  w / g / mom / shadow are the
    range's views of the flat buffers."""
    __slots__ = ("w", "g", "mom", "shadow", "lr_dev", "first_dev", "wd", "momentum", "dampening", "nesterov",
                 "grad_scale", "blocks")

    def __init__(self, w, g, mom, shadow, lr_dev, first_dev, wd, momentum, dampening, nesterov, grad_scale,
                 blocks=128):
        _chk(w, F32, "rider w")
        _chk(g, F32, "rider g")
        if lr_dev is None or w.numel() != g.numel() or (mom is not None and mom.numel() != w.numel()):
            raise ValueError("SgdRider: device lr and matching w / g / mom ranges required")
        self.w, self.g, self.mom, self.shadow = w, g, mom, shadow
        self.lr_dev, self.first_dev = lr_dev, first_dev
        self.wd, self.momentum, self.dampening = float(wd), float(momentum), float(dampening)
        self.nesterov, self.grad_scale, self.blocks = bool(nesterov), float(grad_scale), int(blocks)

    def arm(self):
        """The next rider-capable launch (grouped conv backward, BN backward apply) carries this update."""
        HIP.call("kml_rider_set", "p p p p p p f f f i f l i", _p(self.w), _p(self.g), _p(self.mom),
                 _p(self.shadow), _p(self.lr_dev), _p(self.first_dev), self.wd, self.momentum, self.dampening,
                 int(self.nesterov), self.grad_scale, self.w.numel(), self.blocks)

    def run_alone(self):
        """The same update as its own launch (its host took a path without a rider role)."""
        sgd_(self.w, self.g, self.mom, self.shadow, 0.0, wd=self.wd, momentum=self.momentum,
             dampening=self.dampening, nesterov=self.nesterov, grad_scale=self.grad_scale, lr_dev=self.lr_dev,
             first_dev=self.first_dev, max_blocks=self.blocks)

    @staticmethod
    def disarm():
        """Drop an armed rider (its host launch was not issued)."""
        HIP.call("kml_rider_set", "p p p p p p f f f i f l i", 0, 0, 0, 0, 0, 0, 0.0, 0.0, 0.0, 0, 1.0, 0, 0)


class _Riding:
    """``with _Riding(rider): <one rider-capable launch>``: arm before the launch; afterwards an
    unconsumed rider (the call took a path without a rider role) runs as its own launch; on an
    exception it is dropped."""

    def __init__(self, rider):
        self.rider = rider

    def __enter__(self):
        if self.rider is not None:
            self.rider.arm()
        return self

    def __exit__(self, exc_type, exc, tb):
        if self.rider is not None:
            if exc_type is None:
                HIP.call("kml_rider_flush", "s", _s())
            else:
                SgdRider.disarm()
        return False


def adam_(w, g, m, v, shadow, lr, step, b1=0.9, b2=0.999, eps=1e-8, wd=0.0, decoupled=False,
          grad_scale=1.0, lr_dev=None, step_dev=None, max_blocks=0):
    n = w.numel()
    HIP.call("kml_adam", "p p p p p p p f f f f f f i f l i s", _p(w), _p(g), _p(m), _p(v), _p(shadow),
             _p(lr_dev), _p(step_dev), float(lr), float(step), float(b1), float(b2), float(eps), float(wd),
             int(decoupled), float(grad_scale), n, int(max_blocks), _s())


def increment_(t, by=1.0):
    HIP.call("kml_increment", "p f s", _p(t), float(by), _s())


def clip_grad_norm_(g, ws1, max_norm):
    HIP.call("kml_clip_grad_norm", "p p f l s", _p(g), _p(ws1), float(max_norm), g.numel(), _s())


def kavg_pack_(state, i64, i64_off, n_i64, count_idx, participate):
    """K-AVG round prologue on the flat state buffer (see optim.hip): int64 buffers into
    their fp32 slots, participation flag into the count slot."""
    _chk(state, F32, "state")
    if i64 is not None and (i64.dtype != torch.int64 or not i64.is_contiguous() or i64.numel() < n_i64):
        raise ValueError("kavg_pack_: int64 arena must be contiguous int64 with n_i64 elements")
    if not (0 <= i64_off and i64_off + n_i64 <= count_idx < state.numel()):
        raise ValueError("kavg_pack_: bad state layout")
    HIP.call("kml_kavg_pack", "p p l i l i s", _p(state), _p(i64), int(i64_off), int(n_i64), int(count_idx),
             int(bool(participate)), _s())


def kavg_finish_(state, n_params, count_idx, shadow, i64, i64_off, n_i64):
    """K-AVG round epilogue after the SUM all-reduce: scale by 1/count (device), refresh
    the bf16 shadow of the parameter range, floor the int64 buffers back."""
    _chk(state, F32, "state")
    if shadow is not None and (shadow.dtype != BF16 or shadow.numel() < n_params):
        raise ValueError("kavg_finish_: shadow must be bf16 covering the parameters")
    if not (0 <= n_params <= count_idx < state.numel()):
        raise ValueError("kavg_finish_: bad state layout")
    HIP.call("kml_kavg_finish", "p l l p p l i s", _p(state), int(n_params), int(count_idx), _p(shadow), _p(i64),
             int(i64_off), int(n_i64), _s())


def kavg_snap_(x, flat, snap):
    """flat := x and snap := x (fp32, one pass): the staleness-1 K-AVG round launch."""
    for t, n in ((x, "x"), (flat, "flat"), (snap, "snap")):
        _chk(t, F32, n)
    if not (x.numel() == flat.numel() == snap.numel()):
        raise ValueError("kavg_snap_: size mismatch")
    HIP.call("kml_kavg_snap", "p p p l s", _p(x), _p(flat), _p(snap), x.numel(), _s())


def kavg_async_apply_(x, flat, snap, shadow, world, n_params):
    """x += flat / world - snap (the in-flight average replaces the stale base), the bf16
    shadow of x[:n_params] refreshed in the same pass."""
    for t, n in ((x, "x"), (flat, "flat"), (snap, "snap")):
        _chk(t, F32, n)
    if not (x.numel() == flat.numel() == snap.numel()) or n_params > x.numel():
        raise ValueError("kavg_async_apply_: size mismatch")
    if shadow is not None and (shadow.dtype != BF16 or shadow.numel() < n_params):
        raise ValueError("kavg_async_apply_: shadow must be bf16 covering the parameters")
    HIP.call("kml_kavg_async_apply", "p p p p f l l s", _p(x), _p(flat), _p(snap), _p(shadow), float(world),
             x.numel(), int(n_params), _s())


# --------------------------------------------------------------------------------------
# data
# --------------------------------------------------------------------------------------

def augment(src_u8, labels_src, ctr, B, out=None, labels_out=None, CP=8, pad=4, flip=True, train=True,
            mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225)):
    """src_u8 [N,H,W,C] uint8 on device -> [B,H,W,CP] bf16 normalised batch starting at ctr[2]."""
    N, H, W, C = src_u8.shape
    if out is None:
        out = torch.empty((B, H, W, CP), dtype=BF16, device=src_u8.device)
    if labels_out is None:
        labels_out = torch.empty((B,), dtype=torch.int64, device=src_u8.device)
    mean_a = (torch.tensor(list(mean) + [0.0] * (4 - len(mean)), dtype=F32))
    std_a = (torch.tensor(list(std) + [1.0] * (4 - len(std)), dtype=F32))
    HIP.call("kml_augment", "p p p p p i i i i i i i i i p p s", _p(src_u8), _p(labels_src), _p(out),
             _p(labels_out), _p(ctr), N, H, W, C, CP, B, pad, int(flip), int(train),
             mean_a.data_ptr(), std_a.data_ptr(), _s())
    return out, labels_out


# --------------------------------------------------------------------------------------
# layout / misc
# --------------------------------------------------------------------------------------

def colsum_(x2d, out):
    """out (fp32, [C]) += column sums of bf16 [M, C]."""
    _chk(x2d, BF16, "x")
    C = x2d.shape[-1]
    HIP.call("kml_colsum_bf16", "p p l i s", _p(x2d), _p(out), x2d.numel() // C, C, _s())
    return out


def slab_sum_add_(part, dst):
    """dst (fp32) += part.sum(0) for part [S, *dst.shape] fp32, one pass, slabs in order."""
    _chk(part, F32, "part")
    _chk(dst, F32, "dst")
    n = dst.numel()
    if part.numel() != part.shape[0] * n or n % 4:
        raise ValueError(f"slab_sum_add_: part {tuple(part.shape)} vs dst {tuple(dst.shape)}")
    HIP.call("kml_slab_sum_add", "p p l i s", _p(part), _p(dst), n, part.shape[0], _s())
    return dst


def row_index(pos, L):
    """int64 [B*P]: b * L + pos[b, j] (flat token rows of per-sequence positions), one launch."""
    if pos.dtype != torch.int64 or pos.dim() != 2:
        raise TypeError("row_index: int64 [B, P] positions")
    pos = pos.contiguous()
    B, P = pos.shape
    out = torch.empty(B * P, dtype=torch.int64, device=pos.device)
    HIP.call("kml_row_index", "p p i i l s", _p(pos), _p(out), B, P, int(L), _s())
    return out


def mlm_mask(ids, ctr, P, mask_id=103, vocab=30522, advance=True, out=None):
    """BERT MLM masking on the device (kml_mlm_mask): ids [B, L] int64 -> (masked ids [B, L],
    positions [B, P] ascending, labels [B, P]); P positions per sequence chosen uniformly without
    replacement, 80 % -> mask_id, 10 % -> random token, 10 % kept.  ctr: the [seed, step] fp32
    device tensor; advance: the kernel's last block bumps ctr[1] (fresh masks per replay)."""
    _chk(ids, torch.int64, "ids", 2)
    _chk(ctr, F32, "ctr")
    B, L = ids.shape
    if out is None:
        out = (torch.empty_like(ids), torch.empty((B, P), dtype=torch.int64, device=ids.device),
               torch.empty((B, P), dtype=torch.int64, device=ids.device))
    x, pos, lab = out
    tk = _COUNTERS.take(ids.device, 1) if advance else None
    HIP.call("kml_mlm_mask", "p p p p p p i i i l l s", _p(ids), _p(x), _p(pos), _p(lab), _p(ctr), _p(tk), B, L,
             int(P), int(mask_id), int(vocab), _s())
    return x, pos, lab


def add_i64_(t, v=1):
    HIP.call("kml_add_i64", "p l i s", _p(t), int(v), t.numel(), _s())


def pad_channels(x, CP):
    _chk(x, BF16, "x")
    C = x.shape[-1]
    y = torch.empty(x.shape[:-1] + (CP,), dtype=BF16, device=x.device)
    HIP.call("kml_pad_channels", "p p l i i s", _p(x), _p(y), x.numel() // C, C, CP, _s())
    return y


def nchw_to_nhwc_bf16(x, CP=None):
    """User NCHW fp32 tensor -> NHWC bf16 with channels padded to a multiple of 8."""
    x = x.float().contiguous()
    B, C, H, W = x.shape
    CP = CP or -(-C // 8) * 8
    y = torch.empty((B, H, W, CP), dtype=BF16, device=x.device)
    HIP.call("kml_nchw_to_nhwc_bf16", "p p i i i i s", _p(x), _p(y), B, C, H * W, CP, _s())
    return y


def advance_counter_(ctr, batch, n):
    """ctr = [seed, step, start]: step += 1, start = (start + batch) mod n (device-side)."""
    HIP.call("kml_advance_counter", "p f f s", _p(ctr), float(batch), float(n), _s())
