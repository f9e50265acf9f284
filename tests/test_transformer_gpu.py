"""Numerics of the transformer HIP kernels vs fp32 PyTorch references."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _ref_attn(q, k, v, B, H, L, bias):
    # q,k,v: [B*L, H*64] fp32
    def sp(t):
        return t.view(B, L, H, 64).permute(0, 2, 1, 3)
    s = sp(q) @ sp(k).transpose(-1, -2) / 8.0
    if bias is not None:
        s = s + bias.view(B, 1, 1, L)
    p = s.softmax(-1)
    o = p @ sp(v)
    return o.permute(0, 2, 1, 3).reshape(B * L, H * 64)


@pytest.mark.parametrize("B,H,L,use_bias", [(2, 3, 128, False), (2, 2, 100, True), (1, 12, 512, False),
                                            (3, 1, 64, True), (1, 2, 7, False), (2, 2, 300, True)])
def test_attention_fwd_bwd(B, H, L, use_bias):
    from kubeml_amd.ops import transformer as T
    torch.manual_seed(0)
    qkv = (torch.randn(B * L, 3 * H * 64, device=dev) * 0.5).to(torch.bfloat16)
    q, k, v = qkv[:, :H * 64], qkv[:, H * 64:2 * H * 64], qkv[:, 2 * H * 64:]
    bias = None
    if use_bias:
        keep = torch.rand(B, L, device=dev) > 0.2
        keep[:, 0] = True
        bias = torch.where(keep, 0.0, -10000.0).float().contiguous()
    out, lse = T.attn_fwd(q, k, v, B, H, L, bias=bias)
    qf, kf, vf = (t.float().clone().requires_grad_(True) for t in (q, k, v))
    ref = _ref_attn(qf, kf, vf, B, H, L, bias)
    assert _rel(out, ref) < 1e-2
    dout = torch.randn(B * L, H * 64, device=dev).to(torch.bfloat16)
    ref.backward(dout.float())
    dqkv = torch.empty_like(qkv)
    dq, dk, dv = dqkv[:, :H * 64], dqkv[:, H * 64:2 * H * 64], dqkv[:, 2 * H * 64:]
    T.attn_bwd(q, k, v, out, dout, lse, B, H, L, bias=bias, dq=dq, dk=dk, dv=dv)
    assert _rel(dq, qf.grad) < 3e-2
    assert _rel(dk, kf.grad) < 3e-2
    assert _rel(dv, vf.grad) < 2e-2


@pytest.mark.parametrize("M,N,res", [(300, 768, True), (64, 1024, False), (5, 128, True)])
def test_layernorm_fwd_bwd(M, N, res):
    from kubeml_amd.ops import transformer as T
    torch.manual_seed(1)
    x = (torch.randn(M, N, device=dev) * 2 + 0.3).to(torch.bfloat16)
    r = torch.randn(M, N, device=dev).to(torch.bfloat16) if res else None
    g = torch.rand(N, device=dev) + 0.5
    b = torch.randn(N, device=dev)
    y, xin, mean, rstd = T.ln_fwd(x, g, b, res=r, eps=1e-12)
    xr = (x.float() + (r.float() if res else 0)).requires_grad_(True)
    gr, br = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = F.layer_norm(xr, (N,), gr, br, eps=1e-12)
    assert _rel(y, yr) < 1e-2
    dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
    yr.backward(dy.float())
    dg, db = torch.zeros(N, device=dev), torch.zeros(N, device=dev)
    dx = T.ln_bwd(dy, xin, mean, rstd, g, dg, db)
    assert _rel(dx, xr.grad) < 2e-2
    assert _rel(dg, gr.grad) < 1e-2 and _rel(db, br.grad) < 1e-2
    dg2, db2 = torch.zeros(N, device=dev), torch.zeros(N, device=dev)
    T.ln_bwd(dy, xin, mean, rstd, g, dg2, db2)
    assert torch.equal(dg, dg2) and torch.equal(db, db2)   # deterministic


def test_gelu_dropout():
    from kubeml_amd.ops import transformer as T
    x = torch.randn(4096, 64, device=dev).to(torch.bfloat16)
    xr = x.float().requires_grad_(True)
    yr = F.gelu(xr)
    assert _rel(T.gelu_fwd(x), yr) < 1e-2
    dy = torch.randn_like(x)
    yr.backward(dy.float())
    assert _rel(T.gelu_bwd(dy, x), xr.grad) < 1e-2
    ctr = torch.tensor([7.0, 3.0], device=dev)
    y1 = T.dropout(x, ctr, 11, 0.1)
    y2 = T.dropout(x, ctr, 11, 0.1)
    assert torch.equal(y1, y2)                                  # regenerated mask
    kept = (y1 != 0) | (x == 0)
    frac = 1 - kept.float().mean().item()
    assert 0.08 < frac < 0.12
    assert _rel(y1[kept], x[kept].float() / 0.9) < 1e-2
    ctr[1] += 1
    assert not torch.equal(T.dropout(x, ctr, 11, 0.1), y1)     # new step -> new mask


def test_embedding_and_rows():
    from kubeml_amd.ops import transformer as T
    torch.manual_seed(2)
    V, N, L, B = 1000, 256, 16, 3
    word = torch.randn(V, N, device=dev).to(torch.bfloat16)
    pos = torch.randn(L, N, device=dev).to(torch.bfloat16)
    typ = torch.randn(2, N, device=dev).to(torch.bfloat16)
    ids = torch.randint(0, V, (B * L,), device=dev)
    tt = torch.randint(0, 2, (B * L,), device=dev)
    out = T.embed_fwd(ids, tt, word, pos, typ, L)
    ref = word.float()[ids] + pos.float().repeat(B, 1) + typ.float()[tt]
    assert _rel(out, ref) < 1e-2
    d = torch.randn(B * L, N, device=dev).to(torch.bfloat16)
    dw, dp, dt = torch.zeros(V, N, device=dev), torch.zeros(L, N, device=dev), torch.zeros(2, N, device=dev)
    T.embed_bwd(ids, tt, d, dw, dp, dt, L)          # all three tables: the fused one-pass kernel
    rw = torch.zeros(V, N, device=dev).index_add_(0, ids, d.float())
    assert _rel(dw, rw) < 1e-5
    assert _rel(dp, d.float().view(B, L, N).sum(0)) < 1e-5
    assert _rel(dt, torch.zeros(2, N, device=dev).index_add_(0, tt, d.float())) < 1e-5
    # BERT's shape class (B = 5 tokens per position: the 4-token unroll plus a tail; accumulate into
    # non-zero tables) and the per-table kernels (a table left out)
    V2, N2, L2, B2 = 30522, 768, 64, 5
    ids2 = torch.randint(0, V2, (B2 * L2,), device=dev)
    ids2[:7] = 42                                   # repeated ids: concurrent atomics on one row
    tt2 = torch.randint(0, 2, (B2 * L2,), device=dev)
    d2 = torch.randn(B2 * L2, N2, device=dev).to(torch.bfloat16)
    w0, p0, t0 = torch.randn(V2, N2, device=dev), torch.randn(L2, N2, device=dev), torch.randn(2, N2, device=dev)
    dw, dp, dt = w0.clone(), p0.clone(), t0.clone()
    T.embed_bwd(ids2, tt2, d2, dw, dp, dt, L2)
    assert _rel(dw, w0.clone().index_add_(0, ids2, d2.float())) < 1e-6
    assert _rel(dp, p0 + d2.float().view(B2, L2, N2).sum(0)) < 1e-6
    assert _rel(dt, t0.clone().index_add_(0, tt2, d2.float())) < 1e-6
    dw2 = w0.clone()
    T.embed_bwd(ids2, None, d2, dw2, None, None, L2)   # word table alone: k_embed_bwd_word
    assert _rel(dw2, dw) < 1e-6
    idx = torch.randperm(B * L, device=dev)[:10]
    g = T.gather_rows(out, idx)
    assert torch.equal(g, out[idx])
    dst = torch.zeros_like(out)
    T.scatter_rows(g, idx, dst)
    assert torch.equal(dst[idx], g) and dst.float().abs().sum() == g.float().abs().sum()


def _attn_keep(seed, step, salt, B, H, L, p):
    """Python replica of the kernel's dropout mask (attention.hip Drop::keep)."""
    import numpy as np
    M = np.uint64(0xFFFFFFFF)

    def mul(a, b):
        return (a.astype(np.uint64) * np.uint64(b)) & M

    thr = np.uint64(int(np.float32(p) * np.float32(65536.0)))
    k0 = np.uint64((int(seed) ^ salt) & 0xFFFFFFFF)
    keep = np.zeros((B, H, L, L), dtype=np.float32)
    q = np.arange(L, dtype=np.uint64).reshape(L, 1)
    key = np.arange(L, dtype=np.uint64).reshape(1, L)
    # one full hash per (q, kbase = 64*kb + 4*g), then a one-multiply finaliser per key pair
    kbase = (key & ~np.uint64(63)) + np.uint64(4) * ((key & np.uint64(15)) >> np.uint64(2))
    c = (q * np.uint64((L + 1) // 2) + (kbase >> np.uint64(1))) & M
    off = (key >> np.uint64(1)) - (kbase >> np.uint64(1))
    for b in range(B):
        for h in range(H):
            bh = np.uint64(b * H + h)
            k1 = ((np.uint64(int(step)) * np.uint64(0x632BE5AB)) & M) ^ ((bh * np.uint64(0x5851F42D)) & M)
            hh = mul(np.full_like(c, k0), 0x9E3779B1) ^ mul((np.full_like(c, k1) + np.uint64(0x7F4A7C15)) & M,
                                                            0x85EBCA77) ^ mul(c, 0xC2B2AE3D)
            hh ^= hh >> np.uint64(15)
            hh = mul(hh, 0x2C1B3C6D)
            hh ^= hh >> np.uint64(12)
            hh = mul(hh, 0x297A2D39)
            hh ^= hh >> np.uint64(15)
            hh = (hh + mul(off, 0x9E3779B9)) & M
            hh ^= hh >> np.uint64(16)
            hh = mul(hh, 0x7FEB352D)
            hh ^= hh >> np.uint64(15)
            half = np.where((key & np.uint64(1)) == 1, hh >> np.uint64(16), hh & np.uint64(0xFFFF))
            keep[b, h] = np.where(half >= thr, 1.0 / (1.0 - p), 0.0)
    return torch.from_numpy(keep)


@pytest.mark.parametrize("L", [64, 100, 300])
def test_attention_dropout_matches_masked_reference(L):
    """Fused attention with probability dropout vs fp32 autograd on the same mask
    (forward output, dQ/dK/dV); dropout rate close to p."""
    from kubeml_amd.nn.transformer import _AttnFn, attention_reference
    torch.manual_seed(5)
    B, H, p = 2, 2, 0.25
    D = H * 64
    qkv = (torch.randn(B * L, 3 * D, device="cuda") * 0.5).to(torch.bfloat16)
    ctr = torch.tensor([11.0, 3.0], device="cuda")
    salt = 7919 * 3
    keep = _attn_keep(11, 3, salt, B, H, L, p)
    frac = float((keep == 0).float().mean())
    assert abs(frac - p) < 0.03, frac
    x = qkv.clone().requires_grad_(True)
    out = _AttnFn.apply(x, B, H, L, None, (ctr, salt, p))
    xr = qkv.float().cpu().requires_grad_(True)
    ref = attention_reference(xr, B, H, L, None, keep=keep)
    g = torch.randn_like(ref)
    out.backward(g.to("cuda").to(torch.bfloat16))
    ref.backward(g)
    rel = lambda a, b: float((a.float().cpu() - b).norm() / b.norm())
    assert rel(out.detach(), ref.detach()) < 2e-2
    assert rel(x.grad, xr.grad) < 3e-2


@pytest.mark.parametrize("N,res", [(768, True), (1024, False)])
def test_layernorm_fused_dropout_matches_separate(N, res):
    """LayerNorm(x, residual, dropout=...) with the dropout inside the LN kernels: output
    and the gradients of x (through the mask) and of the residual are bit-identical to a
    separate Dropout followed by the LayerNorm (same counter-hash mask)."""
    from kubeml_amd.nn import transformer as TR
    from kubeml_amd.nn.flat import flatten_module
    torch.manual_seed(2)
    out = []
    old = TR._LN_DROP_FUSE
    try:
        for fuse in (False, True):
            TR._LN_DROP_FUSE = fuse
            torch.manual_seed(3)
            ln = TR.LayerNorm(N, eps=1e-12).to(dev)
            with torch.no_grad():
                ln.weight.uniform_(0.5, 1.5)
                ln.bias.uniform_(-0.2, 0.2)
            flatten_module(ln)
            drop = TR.Dropout(0.1, TR.RNGState(seed=5)).to(dev)
            drop.salt = 1234
            drop.train()
            g = torch.Generator(device=dev).manual_seed(9)
            x = torch.randn(300, N, device=dev, generator=g).to(torch.bfloat16).requires_grad_()
            r = torch.randn(300, N, device=dev, generator=g).to(torch.bfloat16).requires_grad_() if res else None
            y = ln(x, residual=r, dropout=drop)
            dy = torch.randn(300, N, device=dev, generator=g).to(torch.bfloat16)
            y.backward(dy)
            torch.cuda.synchronize()
            out.append((y.detach().clone(), x.grad.clone(), None if r is None else r.grad.clone()))
    finally:
        TR._LN_DROP_FUSE = old
    (ya, gxa, gra), (yb, gxb, grb) = out
    torch.testing.assert_close(yb, ya, rtol=0, atol=0)
    torch.testing.assert_close(gxb, gxa, rtol=0, atol=0)
    if res:
        torch.testing.assert_close(grb, gra, rtol=0, atol=0)
    # the mask really dropped ~p of the elements
    assert 0.05 < float((gxb == 0).float().mean()) < 0.15


@pytest.mark.parametrize("M,N", [(16384, 3072), (300, 72), (7, 1028)])
def test_gelu_bwd_with_bias_colsum(M, N):
    """gelu_bwd(dbias=...) writes the same dx and adds the column sums of dx to dbias (the FFN1
    bias gradient) in the same pass."""
    from kubeml_amd.ops import kernels as K
    from kubeml_amd.ops import transformer as T
    torch.manual_seed(6)
    dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
    x = torch.randn(M, N, device=dev).to(torch.bfloat16)
    ref = T.gelu_bwd(dy, x)
    db = torch.full((N,), 0.5, device=dev)
    dx = T.gelu_bwd(dy, x, dbias=db)
    torch.testing.assert_close(dx, ref, rtol=0, atol=0)
    want = torch.full((N,), 0.5, device=dev)
    K.colsum_(ref, want)
    assert _rel(db, want) < 1e-5


@pytest.mark.parametrize("L", [64, 300])
def test_attention_keep_bits_match_hash(L):
    """The dropout keep bits the forward stores (attention.hip Drop) decode to the Python
    replica of the hashed mask, and the backward that reads them is bit-identical to the
    backward that re-hashes the mask."""
    import numpy as np
    from kubeml_amd.ops import transformer as T
    torch.manual_seed(9)
    B, H, p = 2, 2, 0.25
    D = H * 64
    qkv = (torch.randn(B * L, 3 * D, device="cuda") * 0.5).to(torch.bfloat16)
    q, k, v = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
    ctr = torch.tensor([11.0, 3.0], device="cuda")
    drop = (ctr, 7919 * 3, p)
    kbuf = T.attn_keep_buffer(B, H, L, "cuda")
    out, lse = T.attn_fwd(q, k, v, B, H, L, drop=drop, keep=kbuf)
    nkb = (L + 63) // 64
    w = kbuf.cpu().numpy().view(np.uint64).reshape(B * H, nkb, nkb * 64)
    key = np.arange(L)
    kl = key % 64
    bit = (16 * ((kl // 4) % 4) + 4 * (kl // 16) + kl % 4).astype(np.uint64)
    got = (w[:, (key // 64)[None, :], np.arange(L)[:, None]] >> bit[None, None, :]) & np.uint64(1)
    ref = (_attn_keep(11, 3, 7919 * 3, B, H, L, p) != 0).numpy().reshape(B * H, L, L)
    assert np.array_equal(got.astype(bool), ref)
    dout = torch.randn(B * L, D, device="cuda").to(torch.bfloat16)
    g1 = T.attn_bwd(q, k, v, out, dout, lse, B, H, L, drop=drop, keep=kbuf)
    g2 = T.attn_bwd(q, k, v, out, dout, lse, B, H, L, drop=drop)
    for a, b in zip(g1, g2):
        assert torch.equal(a, b)


def test_mlm_mask_kernel_recipe():
    """kernels.mlm_mask (one HIP kernel) vs BERT's masking recipe: P distinct ascending positions
    per sequence, labels = the original tokens there, the input changed only there, about
    80 / 10 / 10 % [MASK] / random / kept; a fixed counter gives the same mask, an advancing one
    a new mask per call."""
    from kubeml_amd.ops import kernels as K
    B, L, P, V, MASK = 64, 512, 76, 30522, 103
    g = torch.Generator(device="cuda").manual_seed(0)
    ids = torch.randint(1000, V, (B, L), device="cuda", generator=g)
    ctr = torch.tensor([3.0, 0.0], device="cuda")
    x, pos, lab = K.mlm_mask(ids, ctr, P, MASK, V, advance=False)
    x2, pos2, lab2 = K.mlm_mask(ids, ctr, P, MASK, V, advance=True)
    torch.cuda.synchronize()
    assert torch.equal(pos, pos2) and torch.equal(x, x2) and float(ctr[1]) == 1.0
    x3, pos3, _ = K.mlm_mask(ids, ctr, P, MASK, V)
    assert not torch.equal(pos3, pos) and float(ctr[1]) == 2.0
    assert bool((pos[:, 1:] > pos[:, :-1]).all()) and int(pos.min()) >= 0 and int(pos.max()) < L
    assert torch.equal(lab, ids.gather(1, pos))
    changed = x != ids
    sel = torch.zeros_like(changed)
    sel.scatter_(1, pos, True)
    assert not bool((changed & ~sel).any())
    xv = x.gather(1, pos)
    frac_mask = float((xv == MASK).float().mean())
    frac_keep = float((xv == lab).float().mean())
    assert abs(frac_mask - 0.8) < 0.03 and abs(frac_keep - 0.1) < 0.03, (frac_mask, frac_keep)
    # positions uniform over the sequence
    hist = torch.bincount(pos.reshape(-1) // 64, minlength=8).float()
    assert float(hist.max() / hist.min()) < 1.35, hist
