"""Numerics of every HIP kernel against a plain-PyTorch fp32 reference of the same op.

Inputs are rounded to bf16 first, so the reference sees exactly the values the
kernel sees; tolerances cover fp32 accumulation-order differences and the final
bf16 rounding of outputs.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

dev = "cuda"


def _bf(t):
    return t.to(torch.bfloat16)


def _rel(a, b):
    a = a.float()
    b = b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


CONV_CASES = [
    # B, H, W, Cin, Cout, k, stride, pad
    (4, 32, 32, 8, 64, 7, 2, 3),     # ResNet stem (Cin padded 3->8)
    (8, 8, 8, 64, 64, 3, 1, 1),      # layer1
    (8, 8, 8, 64, 128, 3, 2, 1),     # layer2.0.conv1
    (8, 8, 8, 64, 128, 1, 2, 0),     # layer2 downsample
    (8, 4, 4, 128, 128, 3, 1, 1),
    (8, 2, 2, 256, 512, 3, 2, 1),    # layer4.0.conv1 (2x2 -> 1x1)
    (16, 1, 1, 512, 512, 3, 1, 1),   # layer4 (centre tap only)
    (3, 5, 7, 16, 24, 3, 1, 1),      # ragged
    (33, 1, 1, 512, 1000, 1, 1, 0),  # Linear as 1x1 conv (N not multiple of 32)
]


@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(case, variant):
    from kubeml_amd.ops import kernels as K
    B, H, W, Ci, Co, k, s, p = case
    torch.manual_seed(0)
    x = _bf(torch.randn(B, H, W, Ci, device=dev))
    w = _bf(torch.randn(Co, k, k, Ci, device=dev) * (1.0 / (k * k * Ci) ** 0.5))
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=s, padding=p)
    stats = torch.zeros(2 * Co, device=dev)
    M, Nn = B * yr.shape[2] * yr.shape[3], Co
    cfg = lambda mode, m, n, kd: (K.plan_conv(mode, m, n, kd)[:4] + (variant,))
    r0, r1, s0, s1 = K.tap_window(H, W, k, k, s, s, p, p)
    ntap = (r1 - r0) * (s1 - s0)
    y = K.conv_fwd(x, w, k, k, (s, s), (p, p), stats=stats, cfg=cfg("fwd", M, Co, ntap * Ci))
    assert _rel(y.permute(0, 3, 1, 2), yr) < 1e-2
    yf = yr.detach().permute(0, 2, 3, 1).reshape(-1, Co)
    assert torch.allclose(stats[:Co], yf.sum(0), rtol=2e-2, atol=1e-1 * (yf.shape[0] ** 0.5))
    assert _rel(stats[Co:], (yf * yf).sum(0)) < 2e-2
    dy = _bf(torch.randn_like(yr))
    yr.backward(dy.float())
    dyn = dy.permute(0, 2, 3, 1).contiguous()
    dx = K.conv_dgrad(dyn, w, x.shape, k, k, (s, s), (p, p), cfg=cfg("dgrad", B * H * W, Ci, ntap * Co))
    assert _rel(dx.permute(0, 3, 1, 2), xr.grad) < 1e-2
    dw = torch.zeros(Co, k, k, Ci, device=dev)
    K.conv_wgrad(x, dyn, dw, k, k, (s, s), (p, p), cfg=cfg("wgrad", Co, ntap * Ci, M))
    assert _rel(dw.permute(0, 3, 1, 2), wr.grad) < 1e-2


SPLIT_CFGS = [(64, 64, 64, 8, 0), (32, 32, 32, 4, 0), (128, 64, 64, 2, 0), (64, 128, 32, 16, 0), (32, 64, 64, 1, 0),
              (64, 64, 64, 1, 1), (32, 32, 64, 4, 1), (128, 128, 64, 2, 1), (32, 128, 64, 1, 2), (128, 32, 64, 8, 2),
              (64, 32, 64, 3, 1)]


@pytest.mark.parametrize("cfg", SPLIT_CFGS)
def test_conv_splitk_configs(cfg):
    """Every (tile, BK, split-K) path — incl. the last-arriver slab reduction — matches fp32."""
    from kubeml_amd.ops import kernels as K
    torch.manual_seed(2)
    B, H, W, Ci, Co, k, s, p = 16, 4, 4, 128, 256, 3, 1, 1
    x = _bf(torch.randn(B, H, W, Ci, device=dev))
    w = _bf(torch.randn(Co, k, k, Ci, device=dev) * 0.03)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=s, padding=p)
    stats = torch.zeros(2 * Co, device=dev)
    for _ in range(3):  # repeated launches reuse the ticket counters (reset by last arrivers)
        stats.zero_()
        y = K.conv_fwd(x, w, k, k, (s, s), (p, p), stats=stats, cfg=cfg)
        assert _rel(y.permute(0, 3, 1, 2), yr) < 1e-2
    assert _rel(stats[:Co], yr.detach().sum((0, 2, 3))) < 2e-2
    dy = _bf(torch.randn_like(yr))
    yr.backward(dy.float())
    dyn = dy.permute(0, 2, 3, 1).contiguous()
    add = _bf(torch.randn(B, H, W, Ci, device=dev))
    dx = K.conv_dgrad(dyn, w, x.shape, k, k, (s, s), (p, p), addend=add, cfg=cfg)
    assert _rel(dx.permute(0, 3, 1, 2), xr.grad + add.float().permute(0, 3, 1, 2)) < 1e-2
    dw = torch.zeros(Co, k, k, Ci, device=dev)
    K.conv_wgrad(x, dyn, dw, k, k, (s, s), (p, p), cfg=cfg)
    assert _rel(dw.permute(0, 3, 1, 2), wr.grad) < 1e-2


def test_conv_fwd_bias_relu():
    from kubeml_amd.ops import kernels as K
    x = _bf(torch.randn(8, 6, 6, 16, device=dev))
    w = _bf(torch.randn(32, 3, 3, 16, device=dev) * 0.1)
    b = torch.randn(32, device=dev)
    y = K.conv_fwd(x, w, 3, 3, (1, 1), (1, 1), bias=b, relu=True)
    yr = F.relu(F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b, padding=1))
    assert _rel(y.permute(0, 3, 1, 2), yr) < 1e-2


@pytest.mark.parametrize("cfg", [(256, 256, 6, 1, 7), (256, 256, 0, 1, 7), (256, 128, 1, 1, 7), (128, 256, 2, 1, 7),
                                 (128, 128, 3, 1, 7), (128, 128, 4, 1, 7)])
@pytest.mark.parametrize("shape", [(4, 14, 64, 256), (3, 7, 256, 64), (2, 9, 512, 136), (9, 31, 64, 128)])
def test_conv1x1_gemm_route_output_and_stats_rows(cfg, shape):
    """1x1 / stride-1 conv on the MFMA GEMM (kml_gemm_stats): output vs fp32 torch, the per-M-tile
    [sum | sumsq] rows vs the sums of the bf16 output, ragged M (M % BM != 0), with and without bias;
    a ReLU call takes the same-G implicit-GEMM fallback."""
    from kubeml_amd.ops import kernels as K
    B, H, Ci, Co = shape
    torch.manual_seed(5)
    x = _bf(torch.randn(B, H, H, Ci, device=dev))
    w = _bf(torch.randn(Co, 1, 1, Ci, device=dev) * Ci ** -0.5)
    for bias in (None, torch.randn(Co, device=dev)):
        yr = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), bias)
        G = K.conv_fwd_stats_rows(x.shape, Co, 1, 1, (1, 1), (0, 0), cfg=cfg)
        assert G == K.conv_stats_rows(B * H * H, cfg) <= -(-(B * H * H) // cfg[0])
        rows = torch.full((G * 2 * Co,), float("nan"), device=dev)
        y = K.conv_fwd(x, w, 1, 1, (1, 1), (0, 0), bias=bias, stats=rows, stats_part=True, cfg=cfg)
        assert _rel(y.permute(0, 3, 1, 2), yr) < 1e-2
        yf = y.float().reshape(-1, Co)
        r = rows.view(G, 2, Co).sum(0)
        assert torch.allclose(r[0], yf.sum(0), rtol=1e-4, atol=1e-3)
        assert torch.allclose(r[1], (yf * yf).sum(0), rtol=1e-4, atol=1e-3)
        y2 = K.conv_fwd(x, w, 1, 1, (1, 1), (0, 0), bias=bias, cfg=cfg)   # no statistics: kml_gemm
        assert torch.equal(y2, y)
    y3 = K.conv_fwd(x, w, 1, 1, (1, 1), (0, 0), relu=True, cfg=cfg)
    assert _rel(y3.permute(0, 3, 1, 2), F.relu(F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2)))) < 1e-2


@pytest.mark.parametrize("cfg", [(256, 256, 0, 1, 7), (256, 128, 1, 1, 7), (128, 256, 2, 1, 7), (128, 128, 3, 1, 7),
                                 (128, 128, 4, 1, 7)])
@pytest.mark.parametrize("geom", [(4, 14, 64, 128, 3, 1, 1), (2, 15, 128, 64, 3, 2, 1), (2, 9, 64, 72, 1, 2, 0),
                                  (3, 8, 192, 256, 3, 1, 1)])
def test_conv_gemm_gather_route_matches_torch(cfg, geom):
    """Implicit-GEMM forward on the GEMM tiles (kml_gemm_conv_fwd: im2col A gathered per K-tile by the
    DMA stager, padding taps from the zero page): output and BN statistics rows vs fp32 torch, incl.
    stride 2, ragged M, bias."""
    from kubeml_amd.ops import kernels as K
    B, H, Ci, Co, k, s, p = geom
    torch.manual_seed(7)
    x = _bf(torch.randn(B, H, H, Ci, device=dev))
    w = _bf(torch.randn(Co, k, k, Ci, device=dev) * (k * k * Ci) ** -0.5)
    bias = torch.randn(Co, device=dev)
    yr = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), bias, stride=s, padding=p)
    assert K.conv_fwd_plan(Ci, yr.shape[0] * yr.shape[2] * yr.shape[3], Co, k * k * Ci, cfg=cfg,
                           geom=(H, H, k, k, (s, s), (p, p))) == cfg
    G = K.conv_fwd_stats_rows(x.shape, Co, k, k, (s, s), (p, p), cfg=cfg)
    rows = torch.full((G * 2 * Co,), float("nan"), device=dev)
    y = K.conv_fwd(x, w, k, k, (s, s), (p, p), bias=bias, stats=rows, stats_part=True, cfg=cfg)
    assert _rel(y.permute(0, 3, 1, 2), yr) < 1e-2
    yf = y.float().reshape(-1, Co)
    r = rows.view(G, 2, Co).sum(0)
    assert torch.allclose(r[0], yf.sum(0), rtol=1e-4, atol=1e-3)
    assert torch.allclose(r[1], (yf * yf).sum(0), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("route", [("gather", 128, 128, 2, 1), ("gather", 128, 128, 2, 5), ("gather", 256, 128, 0, 3),
                                   ("gather", 128, 256, 0, 2), ("gather", 256, 256, 0, 8)])
@pytest.mark.parametrize("geom", [(4, 14, 64, 128, 3, 1), (2, 15, 64, 72, 3, 2), (3, 7, 136, 64, 3, 1)])
def test_conv_wgrad_gemm_gather_route_matches_torch(route, geom, monkeypatch):
    """Implicit-GEMM weight gradient on the GEMM tiles (kml_gemm_conv_wgrad: im2col(x) gathered per
    K-tile of output pixels, slab split-K, ordered reduce) vs fp32 torch autograd, store and add."""
    from kubeml_amd.ops import kernels as K
    B, H, Ci, Co, k, s = geom
    p = (k - 1) // 2
    torch.manual_seed(9)
    x = _bf(torch.randn(B, H, H, Ci, device=dev))
    w = _bf(torch.randn(Co, k, k, Ci, device=dev) * 0.05)
    wr = w.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.conv2d(x.float().permute(0, 3, 1, 2), wr, stride=s, padding=p)
    dy = _bf(torch.randn_like(yr))
    yr.backward(dy.float())
    dyn = dy.permute(0, 2, 3, 1).contiguous()
    monkeypatch.setitem(K._WGRAD_GEMM, (B * H * H, Co, Ci, k, s), route)
    assert K.wgrad_gemm_route(x.shape, Co, k, k, (s, s), (p, p)) == route
    dw = torch.full((Co, k, k, Ci), float("nan"), device=dev)
    K.conv_wgrad(x, dyn, dw, k, k, (s, s), (p, p), accumulate=False)
    assert _rel(dw.permute(0, 3, 1, 2), wr.grad) < 1e-2
    K.conv_wgrad(x, dyn, dw, k, k, (s, s), (p, p), accumulate=True)
    assert _rel(dw.permute(0, 3, 1, 2), 2 * wr.grad) < 1e-2


@pytest.mark.parametrize("cfg", [(256, 256, 0, 1, 7), (256, 128, 1, 1, 7), (128, 256, 2, 1, 7), (128, 128, 3, 1, 7),
                                 (128, 128, 4, 1, 7)])
@pytest.mark.parametrize("geom", [(4, 14, 64, 128, 3, 1), (3, 7, 136, 64, 3, 1), (2, 9, 72, 192, 3, 1),
                                  (9, 31, 64, 64, 3, 1)])
def test_conv_dgrad_gemm_gather_route_matches_torch(cfg, geom):
    """Implicit-GEMM input gradient on the GEMM tiles (kml_gemm_conv_dgrad, stride 1): dx vs fp32
    torch autograd with a residual addend, and the consumer-BN rows / ReLU mask vs that dx."""
    from kubeml_amd.ops import kernels as K
    B, H, Ci, Co, k, p = geom
    torch.manual_seed(8)
    x = _bf(torch.randn(B, H, H, Ci, device=dev))
    w = _bf(torch.randn(Co, k, k, Ci, device=dev) * (k * k * Co) ** -0.5)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.conv2d(xr, w.float().permute(0, 3, 1, 2), padding=p)
    dy = _bf(torch.randn_like(yr))
    yr.backward(dy.float())
    dyn = dy.permute(0, 2, 3, 1).contiguous()
    add = _bf(torch.randn(B, H, H, Ci, device=dev))
    dx = K.conv_dgrad(dyn, w, x.shape, k, k, (1, 1), (p, p), addend=add, cfg=cfg)
    assert _rel(dx.permute(0, 3, 1, 2), xr.grad + add.float().permute(0, 3, 1, 2)) < 1e-2
    yb = _bf(torch.randn(B, H, H, Ci, device=dev))
    cb = _bf(torch.randn(B, H, H, Ci, device=dev))
    mean, rstd = torch.randn(Ci, device=dev) * 0.1, torch.rand(Ci, device=dev) + 0.5
    dz, (part, G) = K.conv_dgrad(dyn, w, x.shape, k, k, (1, 1), (p, p), addend=add, cfg=cfg,
                                 bnf=(yb, cb, mean, rstd), bnf_mask=True)
    keep = yb.float() > 0
    assert torch.equal(dz, dx * keep)
    dzf = (dx.float() * keep).reshape(-1, Ci)
    r = part.view(G, 2, Ci).sum(0)
    assert torch.allclose(r[0], dzf.sum(0), rtol=1e-4, atol=1e-3)
    assert torch.allclose(r[1], (dzf * ((cb.float() - mean) * rstd).reshape(-1, Ci)).sum(0), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("cfg", [(256, 256, 0, 1, 7), (256, 128, 1, 1, 7), (128, 256, 2, 1, 7), (128, 128, 3, 1, 7),
                                 (128, 128, 4, 1, 7)])
@pytest.mark.parametrize("shape", [(4, 14, 64, 256), (3, 7, 256, 64), (2, 9, 136, 512), (9, 31, 128, 64)])
def test_conv1x1_dgrad_gemm_route_matches_implicit_gemm(cfg, shape):
    """1x1 / stride-1 dgrad on the MFMA GEMM (kml_gemm_dgrad_bnf) against the implicit-GEMM dgrad:
    dx (+ residual addend) vs fp32 torch, the consumer-BN partial rows and the ReLU-masked output."""
    from kubeml_amd.ops import kernels as K
    B, H, Ci, Co = shape
    torch.manual_seed(6)
    dy = _bf(torch.randn(B, H, H, Co, device=dev))
    w = _bf(torch.randn(Co, 1, 1, Ci, device=dev) * Co ** -0.5)
    xs = (B, H, H, Ci)
    y = _bf(torch.randn(xs, device=dev))
    c = _bf(torch.randn(xs, device=dev) * 2 + 0.3)
    mean, rstd = torch.randn(Ci, device=dev) * 0.1, torch.rand(Ci, device=dev) + 0.5
    add = _bf(torch.randn(xs, device=dev))
    ref = torch.einsum("bhwk,kc->bhwc", dy.float(), w.float().view(Co, Ci))
    for addend in (None, add):
        exp = ref + (addend.float() if addend is not None else 0)
        dx = K.conv_dgrad(dy, w, xs, 1, 1, (1, 1), (0, 0), addend=addend, cfg=cfg)
        assert _rel(dx, exp) < 1e-2
        for mask in (False, True):
            dz, (part, G) = K.conv_dgrad(dy, w, xs, 1, 1, (1, 1), (0, 0), addend=addend, cfg=cfg,
                                         bnf=(y, c, mean, rstd), bnf_mask=mask)
            assert G == K.conv_stats_rows(B * H * H, cfg) <= -(-(B * H * H) // cfg[0])
            keep = (y.float() > 0)
            vb = dx.float()
            assert torch.equal(dz, (dx * keep) if mask else dx)
            dzf = (vb * keep).reshape(-1, Ci)
            xh = ((c.float() - mean) * rstd).reshape(-1, Ci)
            r = part.view(G, 2, Ci).sum(0)
            assert torch.allclose(r[0], dzf.sum(0), rtol=1e-4, atol=1e-3)
            assert torch.allclose(r[1], (dzf * xh).sum(0), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("C,M,relu,res", [(64, 4096, True, False), (128, 1000, True, True), (512, 64, False, True),
                                          (2048, 96, True, False), (64, 300000, True, True), (8, 50, False, False),
                                          (1024, 1031, True, False)])
def test_bn_train_fwd_bwd(C, M, relu, res):
    from kubeml_amd.ops import kernels as K
    torch.manual_seed(1)
    x = _bf(torch.randn(M, C, device=dev) * 2 + 0.5)
    r = _bf(torch.randn(M, C, device=dev)) if res else None
    g = torch.rand(C, device=dev) + 0.5
    b = torch.randn(C, device=dev)
    rm = torch.zeros(C, device=dev)
    rv = torch.ones(C, device=dev)
    stats = torch.zeros(2 * C, device=dev)
    K.bn_stats(x, stats)
    mean = torch.empty(C, device=dev)
    rstd = torch.empty(C, device=dev)
    y = K.bn_apply(x, stats, g, b, res=r, save_mean=mean, save_rstd=rstd, run_mean=rm, run_var=rv, relu=relu)
    # reference
    xr = x.float().requires_grad_(True)
    gr = g.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    rmr = torch.zeros(C, device=dev)
    rvr = torch.ones(C, device=dev)
    yr = F.batch_norm(xr, rmr, rvr, gr, br, training=True, momentum=0.1, eps=1e-5)
    if res:
        yr = yr + r.float()
    if relu:
        yr = F.relu(yr)
    assert _rel(y, yr) < 1e-2
    assert torch.allclose(rm, rmr, atol=1e-3) and torch.allclose(rv, rvr, rtol=1e-2, atol=1e-3)
    dy = _bf(torch.randn(M, C, device=dev))
    yr.backward(dy.float())
    dg = torch.zeros(C, device=dev)
    db = torch.zeros(C, device=dev)
    dres = torch.empty_like(x) if res else None
    dx = K.bn_bwd(dy, y if relu else None, x, mean, rstd, g, dg, db, dres=dres)
    assert _rel(dx, xr.grad) < 2e-2
    assert _rel(dg, gr.grad) < 1e-2
    assert _rel(db, br.grad) < 1e-2
    # every reduction mode agrees; the fused and ticket modes are bitwise reproducible
    old = K._BN_REDUCE
    try:
        for mode in ("fused", "ticket", "atomic"):
            K._BN_REDUCE = mode
            dg2, db2 = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
            dg3, db3 = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
            dx2 = K.bn_bwd(dy, y if relu else None, x, mean, rstd, g, dg2, db2)
            K.bn_bwd(dy, y if relu else None, x, mean, rstd, g, dg3, db3)
            assert _rel(dx2, xr.grad) < 2e-2, mode
            assert _rel(dg2, gr.grad) < 1e-2 and _rel(db2, br.grad) < 1e-2, mode
            if mode != "atomic":
                assert torch.equal(dg2, dg3) and torch.equal(db2, db3), mode
    finally:
        K._BN_REDUCE = old


@pytest.mark.parametrize("shape", [(4, 16, 16, 64), (2, 40, 40, 64), (3, 12, 12, 64), (2, 7, 9, 32)])
def test_maxpool_and_gavg(shape):
    """maxpool_bwd's row packing: 2 rows per block (16x16x64), one row over several chunks per
    thread block (40x40), rows that leave threads idle (12x12, 7x9)."""
    from kubeml_amd.ops import kernels as K
    B, C = shape[0], shape[3]
    x = _bf(torch.randn(*shape, device=dev))
    y, idx = K.maxpool_fwd(x, 3, 2, 1)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    assert torch.equal(y.permute(0, 3, 1, 2).float(), yr)
    dy = _bf(torch.randn_like(yr))
    yr.backward(dy.float())
    dx = K.maxpool_bwd(dy.permute(0, 2, 3, 1).contiguous(), idx, x.shape, 3, 2, 1)
    assert _rel(dx.permute(0, 3, 1, 2), xr.grad) < 1e-2
    g = K.gavgpool_fwd(x)
    assert _rel(g, x.float().mean((1, 2))) < 1e-2
    gd = K.gavgpool_bwd(_bf(torch.ones(B, C, device=dev)), x.shape)
    assert torch.allclose(gd.float(), torch.full_like(gd.float(), 1 / (shape[1] * shape[2])), rtol=1e-2)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_cross_entropy(dtype):
    from kubeml_amd.ops import kernels as K
    logits = (torch.randn(37, 1000, device=dev) * 3).to(dtype)
    labels = torch.randint(0, 1000, (37,), device=dev)
    labels[3] = -100
    out3, ws, lab = K.ce_fwd(logits, labels)
    lr = logits.float().requires_grad_(True)
    ref = F.cross_entropy(lr, labels, ignore_index=-100)
    assert abs(out3[0].item() - ref.item()) < 1e-3 * max(1, abs(ref.item()))
    valid = labels != -100
    correct = (lr.argmax(1) == labels)[valid].sum().item()
    assert int(out3[1].item()) == correct and int(out3[2].item()) == int(valid.sum())
    ref.backward()
    go = torch.tensor([2.0], device=dev)
    d = K.ce_bwd(logits, lab, ws, out3, grad_out=go)
    assert _rel(d, 2 * lr.grad) < 1e-2
    # the in-launch fold over many blocks, repeated (its ticket resets itself)
    big = (torch.randn(1030, 1000, device=dev) * 3).to(dtype)
    bl = torch.randint(0, 1000, (1030,), device=dev)
    bl[::7] = -100
    refb = F.cross_entropy(big.float(), bl, ignore_index=-100)
    for _ in range(3):
        o3, _, _ = K.ce_fwd(big, bl)
        assert abs(o3[0].item() - refb.item()) < 1e-3 * max(1, abs(refb.item()))
        assert int(o3[2].item()) == int((bl != -100).sum())


@pytest.mark.parametrize("C,ld", [(30522, 30528), (1000, 1000), (77, 80), (10, 10)])
def test_cross_entropy_padded_rows(C, ld):
    """Vector (16-byte) and scalar CE paths, with logits rows padded past the real classes
    (the MLM decoder's vocab 30522 in a 30528-wide row): loss, argmax count and gradient vs
    torch on the unpadded logits; the gradient's pad columns are zero."""
    from kubeml_amd.ops import kernels as K
    torch.manual_seed(3)
    B = 45
    full = (torch.randn(B, ld, device=dev) * 3).to(torch.bfloat16)
    labels = torch.randint(0, C, (B,), device=dev)
    labels[5] = -100
    out3, ws, lab = K.ce_fwd(full, labels, classes=C)
    lr = full[:, :C].float().requires_grad_(True)
    ref = F.cross_entropy(lr, labels, ignore_index=-100)
    assert abs(out3[0].item() - ref.item()) < 1e-3 * max(1, abs(ref.item()))
    valid = labels != -100
    assert int(out3[1].item()) == int((lr.argmax(1) == labels)[valid].sum().item())
    ref.backward()
    d = K.ce_bwd(full, lab, ws, out3, classes=C)
    assert _rel(d[:, :C], lr.grad) < 1e-2
    if ld > C:
        assert float(d[:, C:].float().abs().max()) == 0.0


def test_sgd_adam():
    from kubeml_amd.ops import kernels as K
    n = 10007
    w = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev)
    mom = torch.zeros(n, device=dev)
    sh = torch.empty(n, dtype=torch.bfloat16, device=dev)
    wr = w.clone().requires_grad_(False)
    opt = torch.optim.SGD([torch.nn.Parameter(wr)], lr=0.1, momentum=0.9, weight_decay=1e-4)
    p = opt.param_groups[0]["params"][0]
    for it in range(3):
        p.grad = g.clone()
        opt.step()
        K.sgd_(w, g, mom, sh, 0.1, wd=1e-4, momentum=0.9, first=(it == 0))
    assert torch.allclose(w, p.data, atol=1e-5)
    assert torch.allclose(sh.float(), w, rtol=1e-2, atol=1e-2)
    # adamw
    w2 = torch.randn(n, device=dev)
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    p2 = torch.nn.Parameter(w2.clone())
    opt2 = torch.optim.AdamW([p2], lr=1e-3, weight_decay=0.01)
    for it in range(3):
        p2.grad = g.clone()
        opt2.step()
        K.adam_(w2, g, m, v, None, 1e-3, it + 1, wd=0.01, decoupled=True)
    assert torch.allclose(w2, p2.data, atol=1e-5)



def test_sgd_folds_the_data_counter_advance():
    """sgd_(advance=(ctr, B, n)): identical update, and ctr ends where advance_counter_
    leaves it (step + 1, start + B wrapped at n), over launches that wrap around."""
    from kubeml_amd.ops import kernels as K
    n = 10007
    w1 = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev)
    w2 = w1.clone()
    s1 = torch.empty(n, dtype=torch.bfloat16, device=dev)
    s2 = torch.empty_like(s1)
    c1 = torch.tensor([3.0, 0.0, 0.0], device=dev)
    c2 = c1.clone()
    for _ in range(7):
        K.sgd_(w1, g, None, s1, 0.05, wd=1e-4)
        K.advance_counter_(c1, 48, 100)
        K.sgd_(w2, g, None, s2, 0.05, wd=1e-4, advance=(c2, 48, 100))
    assert torch.equal(w2, w1) and torch.equal(s2, s1)
    assert torch.equal(c2, c1) and c2.tolist() == [3.0, 7.0, 36.0]

def test_augment():
    from kubeml_amd.ops import kernels as K
    N = 50
    src = torch.randint(0, 256, (N, 32, 32, 3), dtype=torch.uint8, device=dev)
    lab = torch.randint(0, 10, (N,), device=dev)
    ctr = torch.tensor([7.0, 3.0, 40.0], device=dev)
    out, lo = K.augment(src, lab, ctr, 16, train=False)
    mean = torch.tensor([0.485, 0.456, 0.406], device=dev)
    std = torch.tensor([0.229, 0.224, 0.225], device=dev)
    idx = (torch.arange(16, device=dev) + 40) % N
    ref = (src[idx].float() / 255 - mean) / std
    assert _rel(out[..., :3], ref) < 1e-2
    assert (out[..., 3:] == 0).all()
    assert torch.equal(lo, lab[idx])
    out2, _ = K.augment(src, lab, ctr, 16, train=True)
    assert out2.shape == (16, 32, 32, 8)


@pytest.mark.parametrize("B,H,W,ci,co,k", [(32, 1, 1, 88, 16, 1), (32, 1, 1, 120, 88, 1), (8, 6, 6, 8, 8, 3),
                                           (4, 5, 5, 16, 24, 3)])
def test_conv_outputs_stay_in_bounds(B, H, W, ci, co, k):
    """Every mode writes only its own output: a guard band after the output / weight
    gradient must stay untouched (tiles larger than M or N, split-K, atomics)."""
    from kubeml_amd.ops import kernels as K
    torch.manual_seed(3)
    p = k // 2
    OH, OW = K.out_hw(H, W, k, k, 1, 1, p, p)
    x = _bf(torch.randn(B, H, W, ci, device=dev))
    w = _bf(torch.randn(co, k, k, ci, device=dev) * 0.1)
    dy = _bf(torch.randn(B, OH, OW, co, device=dev))
    GUARD = 4096
    for cfg in [None, (32, 32, 32, 1, 0), (64, 64, 64, 1, 0), (32, 32, 64, 4, 0), (64, 32, 64, 2, 1),
                (128, 128, 64, 1, 2)]:
        wbuf = torch.zeros(co * k * k * ci + GUARD, device=dev)
        dw = wbuf[:co * k * k * ci].view(co, k, k, ci)
        K.conv_wgrad(x, dy, dw, k, k, (1, 1), (p, p), cfg=cfg)
        assert wbuf[co * k * k * ci:].abs().max().item() == 0.0, ("wgrad", cfg)
        ybuf = torch.zeros(B * OH * OW * co + GUARD, dtype=torch.bfloat16, device=dev)
        y = ybuf[:B * OH * OW * co].view(B, OH, OW, co)
        K.conv_fwd(x, w, k, k, (1, 1), (p, p), out=y, cfg=cfg)
        assert ybuf[B * OH * OW * co:].float().abs().max().item() == 0.0, ("fwd", cfg)
        xbuf = torch.zeros(B * H * W * ci + GUARD, dtype=torch.bfloat16, device=dev)
        dx = xbuf[:B * H * W * ci].view(B, H, W, ci)
        K.conv_dgrad(dy, w, x.shape, k, k, (1, 1), (p, p), out=dx, cfg=cfg)
        assert xbuf[B * H * W * ci:].float().abs().max().item() == 0.0, ("dgrad", cfg)


@pytest.mark.parametrize("shape", [(16, 4, 4, 128, 256, 3, 1, 1), (8, 8, 8, 64, 128, 3, 2, 1),
                                   (32, 1, 1, 512, 512, 3, 1, 1), (8, 4, 4, 96, 40, 3, 1, 1),
                                   (16, 2, 2, 256, 512, 1, 2, 0)])
@pytest.mark.parametrize("tile", [(16, 16, 4), (32, 32, 8), (64, 32, 4), (32, 64, 8)])
def test_conv_direct_variant(shape, tile):
    """LDS-free wave-split-K kernel (variant 3): fwd (+bias/ReLU/BN stats) and dgrad
    (+ transposed weights, + fused addend) vs fp32 torch."""
    from kubeml_amd.ops import kernels as K
    B, H, W, Ci, Co, k, s, p = shape
    bm, bn, nw = tile
    cfg = (bm, bn, nw, 1, 3)
    torch.manual_seed(4)
    x = _bf(torch.randn(B, H, W, Ci, device=dev))
    w = _bf(torch.randn(Co, k, k, Ci, device=dev) * 0.05)
    bias = torch.randn(Co, device=dev)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.float().permute(0, 3, 1, 2)
    pre = F.conv2d(xr, wr, bias, stride=s, padding=p)
    yr = F.relu(pre)
    stats = torch.zeros(2 * Co, device=dev)
    y = K.conv_fwd(x, w, k, k, (s, s), (p, p), bias=bias, stats=stats, relu=True, cfg=cfg)
    assert _rel(y.permute(0, 3, 1, 2), yr) < 1e-2
    assert _rel(stats[:Co], yr.detach().sum((0, 2, 3))) < 2e-2
    dy = _bf(torch.randn_like(pre))
    pre.backward(dy.float())
    add = _bf(torch.randn(B, H, W, Ci, device=dev))
    dx = K.conv_dgrad(dy.permute(0, 2, 3, 1).contiguous(), w, x.shape, k, k, (s, s), (p, p), addend=add, cfg=cfg)
    assert _rel(dx.permute(0, 3, 1, 2), xr.grad + add.float().permute(0, 3, 1, 2)) < 1e-2


HALO_CASES = [(4, 8, 64, 64), (3, 8, 64, 128), (6, 4, 128, 128), (5, 4, 128, 256), (2, 8, 256, 64),
              (3, 4, 256, 64), (2, 4, 512, 64)]


@pytest.mark.parametrize("case", HALO_CASES)
def test_conv_halo_variant(case):
    """Halo-patch forward (variant 4: whole zero-padded images staged in LDS once, weights
    streamed into MFMA registers) for every instantiated tile: output (+bias/ReLU), atomic
    statistics and per-M-tile partial rows vs fp32 torch; batches that do not fill the last
    block's images exercise the zero-page tail."""
    from kubeml_amd.ops import kernels as K
    B, H, Ci, Co = case
    torch.manual_seed(11)
    x = _bf(torch.randn(B, H, H, Ci, device=dev))
    w = _bf(torch.randn(Co, 3, 3, Ci, device=dev) * (1.0 / (9 * Ci) ** 0.5))
    bias = torch.randn(Co, device=dev)
    pre = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), bias, padding=1)
    tiles = [t for t in K._HALO_TILES[(Ci, H)] if Co % t[1] == 0]
    assert tiles and K.halo_plan(Ci, Co, H, H, 3, 3, (1, 1), (1, 1)) is not None
    for bm, bn in tiles:
        cfg = (bm, bn, 0, 1, K.HALO)
        st = torch.zeros(2 * Co, device=dev)
        y = K.conv_fwd(x, w, 3, 3, (1, 1), (1, 1), bias=bias, stats=st, relu=True, cfg=cfg)
        yr = F.relu(pre)
        assert _rel(y.permute(0, 3, 1, 2), yr) < 1e-2, (bm, bn)
        assert _rel(st[:Co], yr.sum((0, 2, 3))) < 2e-2, (bm, bn)
        G = K.conv_fwd_stats_rows(x.shape, Co, 3, 3, (1, 1), (1, 1), cfg=cfg)
        assert G == -(-B * H * H // bm)
        buf = torch.full((G * 2 * Co + 256,), float("nan"), device=dev)
        y2 = K.conv_fwd(x, w, 3, 3, (1, 1), (1, 1), stats=buf[:G * 2 * Co], stats_part=True, cfg=cfg)
        assert torch.isnan(buf[G * 2 * Co:]).all() and not torch.isnan(buf[:G * 2 * Co]).any()
        yf = (pre - bias.view(1, -1, 1, 1))
        assert _rel(y2.permute(0, 3, 1, 2), yf) < 1e-2, (bm, bn)
        rows = buf[:G * 2 * Co].view(G, 2, Co).sum(0)
        assert _rel(rows[0], yf.sum((0, 2, 3))) < 2e-2 and _rel(rows[1], (yf * yf).sum((0, 2, 3))) < 2e-2


@pytest.mark.parametrize("case", [(4, 8, 64, 64), (3, 8, 128, 64), (6, 4, 128, 128), (5, 4, 256, 128)])
def test_conv_halo_dgrad(case, monkeypatch):
    """Halo-patch dgrad (variant 4: padded dy patch in LDS, flipped-filter weight slice read
    with transposing LDS reads): dx (+ residual addend) vs fp32 torch, and the consumer-BN
    fusion (masked dz + dgamma/dbeta partial rows) vs the implicit-GEMM plan."""
    from kubeml_amd.ops import kernels as K
    monkeypatch.setattr(K, "_HALO_DG_ON", True)      # opt-in in the step (profiles/r3/halo_dgrad.md)
    B, H, Ci, Co = case
    torch.manual_seed(12)
    x = _bf(torch.randn(B, H, H, Ci, device=dev))
    w = _bf(torch.randn(Co, 3, 3, Ci, device=dev) * (1.0 / (9 * Ci) ** 0.5))
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.conv2d(xr, wr, padding=1)
    dy = _bf(torch.randn_like(yr))
    yr.backward(dy.float())
    dyn = dy.permute(0, 2, 3, 1).contiguous()
    add = _bf(torch.randn(B, H, H, Ci, device=dev))
    # the step's grouped backward (halo dgrad + wgrad in one launch when instantiated)
    dplan, wplan, grouped = K.bwd_plans(x.shape, Co, 3, 3, (1, 1), (1, 1))
    assert dplan[4] == K.HALO
    dw = torch.full((Co, 3, 3, Ci), float("nan"), device=dev)
    dx = K.conv_bwd(dyn, w, x, dw, 3, 3, (1, 1), (1, 1), addend=add, accumulate=False)
    assert _rel(dx.permute(0, 3, 1, 2), xr.grad + add.float().permute(0, 3, 1, 2)) < 1e-2, grouped
    assert _rel(dw.permute(0, 3, 1, 2), wr.grad) < 1e-2, grouped
    c = _bf(torch.randn(B, H, H, Ci, device=dev))
    yb = _bf(torch.randn(B, H, H, Ci, device=dev))
    mean, rstd = torch.randn(Ci, device=dev) * 0.1, torch.rand(Ci, device=dev) + 0.5
    tiles = [t for t in K._HALO_DG_TILES[(Co, H)] if Ci % t[1] == 0]
    assert tiles and K.halo_dgrad_plan(Ci, Co, H, H, 3, 3, (1, 1), (1, 1)) is not None
    base = K.plan_conv("dgrad", B * H * H, Ci, 9 * Co)
    r_ref = K.conv_dgrad(dyn, w, x.shape, 3, 3, (1, 1), (1, 1), cfg=base, bnf=(yb, c, mean, rstd), bnf_mask=True)
    for bm, bn in tiles:
        cfg = (bm, bn, 0, 1, K.HALO)
        dx = K.conv_dgrad(dyn, w, x.shape, 3, 3, (1, 1), (1, 1), addend=add, cfg=cfg)
        assert _rel(dx.permute(0, 3, 1, 2), xr.grad + add.float().permute(0, 3, 1, 2)) < 1e-2, (bm, bn)
        r = K.conv_dgrad(dyn, w, x.shape, 3, 3, (1, 1), (1, 1), cfg=cfg, bnf=(yb, c, mean, rstd), bnf_mask=True)
        assert _rel(r[0], r_ref[0]) < 1e-2, (bm, bn)
        (p1, g1), (p0, g0) = r[1], r_ref[1]
        assert g1 == -(-B * H * H // bm)
        assert _rel(p1.view(g1, 2 * Ci).sum(0), p0.view(g0, 2 * Ci).sum(0)) < 2e-2, (bm, bn)


@pytest.mark.parametrize("cfg", [(32, 32, 64, 1, 0), (64, 32, 64, 2, 1), (128, 64, 64, 1, 2), (32, 32, 4, 1, 3),
                                 (64, 64, 32, 4, 0)])
def test_conv_partial_stats_into_bn_apply(cfg):
    """FWD epilogue partial statistics (plain stores per wave row-band) summed by bn_apply
    equal the atomic statistics; M not a multiple of the tile exercises the tail rows."""
    from kubeml_amd.ops import kernels as K
    torch.manual_seed(5)
    B, H, W, Ci, Co = 7, 5, 5, 64, 96   # M = 175
    x = _bf(torch.randn(B, H, W, Ci, device=dev))
    w = _bf(torch.randn(Co, 3, 3, Ci, device=dev) * 0.05)
    st_a = torch.zeros(2 * Co, device=dev)
    y = K.conv_fwd(x, w, 3, 3, (1, 1), (1, 1), stats=st_a, cfg=cfg)
    G = K.conv_fwd_stats_rows(x.shape, Co, 3, 3, (1, 1), (1, 1), cfg=cfg)
    guard = 1024
    buf = torch.full((G * 2 * Co + guard,), float("nan"), device=dev)
    y2 = K.conv_fwd(x, w, 3, 3, (1, 1), (1, 1), stats=buf[:G * 2 * Co], stats_part=True, cfg=cfg)
    assert torch.isnan(buf[G * 2 * Co:]).all()            # nothing written past the G rows
    assert not torch.isnan(buf[:G * 2 * Co]).any()        # every row written
    assert torch.equal(y, y2)
    assert _rel(buf[:G * 2 * Co].view(G, 2 * Co).sum(0), st_a) < 1e-5
    g, b = torch.rand(Co, device=dev) + 0.5, torch.randn(Co, device=dev)
    m1, r1 = torch.empty(Co, device=dev), torch.empty(Co, device=dev)
    m2, r2 = torch.empty(Co, device=dev), torch.empty(Co, device=dev)
    o1 = K.bn_apply(y, st_a, g, b, save_mean=m1, save_rstd=r1, relu=True)
    o2 = K.bn_apply(y, buf, g, b, save_mean=m2, save_rstd=r2, relu=True, stats_rows=G)
    assert _rel(m2, m1) < 1e-5 and _rel(r2, r1) < 1e-5 and _rel(o2, o1) < 1e-2


@pytest.mark.parametrize("M,C", [(65536, 64), (1000, 128), (37, 512)])
def test_bn_stats_partial_rows(M, C):
    from kubeml_amd.ops import kernels as K
    torch.manual_seed(6)
    x = _bf(torch.randn(M, C, device=dev) * 1.5 + 0.2)
    part, G = K.bn_stats_part(x)
    s = part.view(G, 2 * C).sum(0)
    xf = x.float()
    assert _rel(s[:C], xf.sum(0)) < 1e-4 and _rel(s[C:], (xf * xf).sum(0)) < 1e-4


@pytest.mark.parametrize("cfg,Ci,with_add", [
    ((32, 32, 64, 1, 0), 64, True), ((64, 32, 64, 2, 1), 64, True), ((32, 32, 4, 1, 3), 64, True),
    ((64, 64, 32, 4, 0), 64, True),
    # 64-column tiles run the LDS row-pass epilogue (16-byte addend / y / c rows)
    ((64, 64, 32, 1, 0), 192, True), ((64, 64, 32, 1, 0), 192, False), ((64, 64, 64, 1, 0), 64, False),
    ((64, 128, 64, 1, 1), 192, True), ((64, 128, 64, 1, 1), 64, False)])
def test_dgrad_emits_consumer_bn_partials(cfg, Ci, with_add):
    """conv_dgrad(bnf=...) writes the dgamma/dbeta partial rows of the BN that consumes dX;
    bn_bwd(partial=...) then equals the unfused bn_bwd."""
    from kubeml_amd.ops import kernels as K
    torch.manual_seed(7)
    B, H, W, Co = 6, 5, 5, 96
    dy = _bf(torch.randn(B, H, W, Co, device=dev))
    w = _bf(torch.randn(Co, 3, 3, Ci, device=dev) * 0.05)
    add = _bf(torch.randn(B, H, W, Ci, device=dev)) if with_add else None
    c = _bf(torch.randn(B, H, W, Ci, device=dev))            # the consumer BN's input
    ybn = _bf(torch.randn(B, H, W, Ci, device=dev))          # its ReLU output (sign pattern)
    mean, rstd = torch.randn(Ci, device=dev), torch.rand(Ci, device=dev) + 0.5
    g = torch.rand(Ci, device=dev) + 0.5
    dx0 = K.conv_dgrad(dy, w, (B, H, W, Ci), 3, 3, (1, 1), (1, 1), addend=add, cfg=cfg)
    dx1, partial = K.conv_dgrad(dy, w, (B, H, W, Ci), 3, 3, (1, 1), (1, 1), addend=add, cfg=cfg,
                                bnf=(ybn, c, mean, rstd))
    assert torch.equal(dx0, dx1)
    dg0, db0 = torch.zeros(Ci, device=dev), torch.zeros(Ci, device=dev)
    dg1, db1 = torch.zeros(Ci, device=dev), torch.zeros(Ci, device=dev)
    r0 = K.bn_bwd(dx0, ybn, c, mean, rstd, g, dg0, db0)
    r1 = K.bn_bwd(dx1, ybn, c, mean, rstd, g, dg1, db1, partial=partial)
    assert _rel(db1, db0) < 1e-4 and _rel(dg1, dg0) < 1e-4
    assert _rel(r1, r0) < 1e-2
    xr = torch.zeros(B, Ci, H, W, device=dev, requires_grad=True)
    F.conv2d(xr, w.float().permute(0, 3, 1, 2), padding=1).backward(dy.float().permute(0, 3, 1, 2))
    ref = xr.grad.permute(0, 2, 3, 1) + (add.float() if add is not None else 0.0)
    assert _rel(dx1, ref) < 1e-2
    # bnf_mask: the dgrad writes dz = dX * [y > 0] itself; the BN backward then runs without
    # y (no mask, y never read) and gives the same dx / dres / dgamma / dbeta
    dz, partial2 = K.conv_dgrad(dy, w, (B, H, W, Ci), 3, 3, (1, 1), (1, 1), addend=add, cfg=cfg,
                                bnf=(ybn, c, mean, rstd), bnf_mask=True)
    assert torch.equal(dz, torch.where(ybn > 0, dx1, torch.zeros_like(dx1)))
    assert torch.equal(partial2[0], partial[0])
    dg2, db2 = torch.zeros(Ci, device=dev), torch.zeros(Ci, device=dev)
    res1, res2 = torch.empty_like(dx1), torch.empty_like(dx1)
    dg3, db3 = torch.zeros(Ci, device=dev), torch.zeros(Ci, device=dev)
    r3 = K.bn_bwd(dx1, ybn, c, mean, rstd, g, dg3, db3, dres=res1, partial=partial)
    r2 = K.bn_bwd(dz, None, c, mean, rstd, g, dg2, db2, dres=res2, partial=partial2)
    assert torch.equal(r2, r3) and torch.equal(res2, res1)
    assert torch.equal(dg2, dg3) and torch.equal(db2, db3)


PAIR_PLANS = [  # (dgrad plan, wgrad plan) pairs with a grouped kernel
    ((32, 64, 64, 1, 0), (32, 32, 64, 1, 0)), ((32, 32, 64, 2, 0), (64, 32, 64, 4, 0)),
    ((32, 32, 4, 1, 3), (32, 32, 64, 2, 0)), ((64, 32, 4, 1, 3), (64, 32, 64, 1, 0)),
    ((32, 16, 4, 1, 3), (32, 32, 64, 8, 0)),
]


@pytest.mark.parametrize("plans", PAIR_PLANS)
@pytest.mark.parametrize("shape", [(8, 8, 8, 64, 64, 3, 1, 1), (6, 5, 5, 64, 96, 3, 1, 1), (8, 8, 8, 64, 128, 3, 2, 1),
                                   (32, 1, 1, 512, 512, 3, 1, 1), (16, 4, 4, 128, 256, 1, 2, 0)])
def test_conv_bwd_pair_matches_separate(plans, shape):
    """Grouped dgrad+wgrad launch (k_conv_pair) == the two separate kernels (bit-exact dX and
    consumer-BN partials; dW equal up to atomic ordering) and the fp32 torch reference."""
    from kubeml_amd.ops import kernels as K
    dcfg, wcfg = plans
    assert K.conv_pair_supported(dcfg, wcfg)
    B, H, W, Ci, Co, k, s, p = shape
    torch.manual_seed(8)
    x = _bf(torch.randn(B, H, W, Ci, device=dev))
    w = _bf(torch.randn(Co, k, k, Ci, device=dev) * 0.05)
    OH, OW = K.out_hw(H, W, k, k, s, s, p, p)
    dy = _bf(torch.randn(B, OH, OW, Co, device=dev))
    add = _bf(torch.randn(B, H, W, Ci, device=dev))
    c = _bf(torch.randn(B, H, W, Ci, device=dev))
    ybn = _bf(torch.randn(B, H, W, Ci, device=dev))
    mean, rstd = torch.randn(Ci, device=dev), torch.rand(Ci, device=dev) + 0.5
    bnf = (ybn, c, mean, rstd)
    dw0 = torch.zeros(Co, k, k, Ci, device=dev)
    K.conv_wgrad(x, dy, dw0, k, k, (s, s), (p, p), cfg=wcfg)
    dx0, (part0, G0) = K.conv_dgrad(dy, w, x.shape, k, k, (s, s), (p, p), addend=add, cfg=dcfg, bnf=bnf)
    dw1 = torch.zeros_like(dw0)
    wt = None
    if dcfg[4] == K.DIRECT:
        wt = torch.empty(Ci, k, k, -(-Co // 32) * 32, dtype=torch.bfloat16, device=dev)
        K.weight_transpose_multi([w], [wt])
    dx1, (part1, G1) = K.conv_bwd(dy, w, x, dw1, k, k, (s, s), (p, p), addend=add, bnf=bnf, wt=wt,
                                  dcfg=dcfg, wcfg=wcfg)
    torch.cuda.synchronize()
    assert torch.equal(dx0, dx1)
    assert G0 == G1 and torch.equal(part0, part1)
    assert _rel(dw1, dw0) < 1e-5
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.float().permute(0, 3, 1, 2).requires_grad_(True)
    F.conv2d(xr, wr, stride=s, padding=p).backward(dy.float().permute(0, 3, 1, 2))
    assert _rel(dw1.permute(0, 3, 1, 2), wr.grad) < 1e-2
    assert _rel(dx1.permute(0, 3, 1, 2), xr.grad + add.float().permute(0, 3, 1, 2)) < 1e-2


def test_weight_transpose_multi():
    from kubeml_amd.ops import kernels as K
    torch.manual_seed(9)
    ws = [_bf(torch.randn(co, k, k, ci, device=dev)) for co, k, ci in [(64, 3, 64), (40, 3, 96), (512, 1, 256)]]
    wts = [torch.full((w.shape[3], w.shape[1], w.shape[2], -(-w.shape[0] // 32) * 32), 7.0, dtype=torch.bfloat16,
                      device=dev) for w in ws]
    K.weight_transpose_multi(ws, wts)
    for w, wt in zip(ws, wts):
        Co = w.shape[0]
        assert torch.equal(wt[..., :Co], w.permute(3, 1, 2, 0))
        assert (wt[..., Co:] == 0).all()


@pytest.mark.parametrize("cfg", [(128, 32, 64, 1, 1), (32, 64, 64, 1, 0), (64, 32, 64, 2, 0), (32, 32, 4, 1, 3)])
def test_grouped_partial_rows(cfg):
    """Large-M convs group-reduce their partial BN rows in the epilogue (last arriver of each
    M-tile group): the consumer sees <= 16 rows whose sum equals the atomic statistics, and
    the dgrad consumer-BN partials give the same dgamma/dbeta as the unfused BN backward."""
    from kubeml_amd.ops import kernels as K
    old_min = K._GRP_MIN
    K._GRP_MIN = 64
    try:
        _grouped_partial_rows(K, cfg)
    finally:
        K._GRP_MIN = old_min


def _grouped_partial_rows(K, cfg):
    torch.manual_seed(10)
    B, H, W, Ci, Co = 256, 8, 8, 64, 64     # M = 16384: well above the grouping threshold
    x = _bf(torch.randn(B, H, W, Ci, device=dev))
    w = _bf(torch.randn(Co, 3, 3, Ci, device=dev) * 0.05)
    G = K.conv_fwd_stats_rows(x.shape, Co, 3, 3, (1, 1), (1, 1), cfg=cfg)
    assert G <= 16
    st_a = torch.zeros(2 * Co, device=dev)
    y = K.conv_fwd(x, w, 3, 3, (1, 1), (1, 1), stats=st_a, cfg=cfg)
    for _ in range(3):   # repeated launches: the group tickets must reset themselves
        buf = torch.full((G * 2 * Co,), float("nan"), device=dev)
        y2 = K.conv_fwd(x, w, 3, 3, (1, 1), (1, 1), stats=buf, stats_part=True, cfg=cfg)
        assert torch.equal(y, y2)
        assert _rel(buf.view(G, 2 * Co).sum(0), st_a) < 1e-5
    dy = _bf(torch.randn(B, H, W, Co, device=dev))
    c = _bf(torch.randn(B, H, W, Ci, device=dev))
    ybn = _bf(torch.randn(B, H, W, Ci, device=dev))
    mean, rstd = torch.randn(Ci, device=dev), torch.rand(Ci, device=dev) + 0.5
    g = torch.rand(Ci, device=dev) + 0.5
    dx1, partial = K.conv_dgrad(dy, w, x.shape, 3, 3, (1, 1), (1, 1), cfg=cfg, bnf=(ybn, c, mean, rstd))
    assert partial[1] <= 16
    dg0, db0 = torch.zeros(Ci, device=dev), torch.zeros(Ci, device=dev)
    dg1, db1 = torch.zeros(Ci, device=dev), torch.zeros(Ci, device=dev)
    r0 = K.bn_bwd(dx1, ybn, c, mean, rstd, g, dg0, db0)
    r1 = K.bn_bwd(dx1, ybn, c, mean, rstd, g, dg1, db1, partial=partial)
    assert _rel(db1, db0) < 1e-4 and _rel(dg1, dg0) < 1e-4
    assert _rel(r1, r0) < 1e-2


LARGE_TILE_CFGS = [(128, 128, 64, 1, 0), (128, 128, 64, 1, 1), (128, 64, 32, 2, 0), (64, 128, 64, 1, 1),
                   (256, 128, 64, 1, 1), (128, 256, 64, 1, 1)]


@pytest.mark.parametrize("cfg", LARGE_TILE_CFGS)
@pytest.mark.parametrize("shape", [(4, 16, 16, 64, 128, 3, 1, 1), (300, 1, 1, 256, 136, 1, 1, 0)])
def test_conv_large_tiles(cfg, shape):
    """Tiles of >= 8192 outputs stage the bf16 output through LDS (16-byte row stores), the
    256-wide LDS-DMA tiles, and the one-row-per-tile BN partials, vs fp32 torch."""
    from kubeml_amd.ops import kernels as K
    B, H, W, Ci, Co, k, s, p = shape
    torch.manual_seed(11)
    x = _bf(torch.randn(B, H, W, Ci, device=dev))
    w = _bf(torch.randn(Co, k, k, Ci, device=dev) * 0.05)
    bias = torch.randn(Co, device=dev)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.float().permute(0, 3, 1, 2).requires_grad_(True)
    pre = F.conv2d(xr, wr, bias, stride=s, padding=p)
    y = K.conv_fwd(x, w, k, k, (s, s), (p, p), bias=bias, cfg=cfg)
    assert _rel(y.permute(0, 3, 1, 2), pre) < 1e-2
    G = K.conv_fwd_stats_rows(x.shape, Co, k, k, (s, s), (p, p), cfg=cfg)
    st = torch.full((G * 2 * Co,), float("nan"), device=dev)
    K.conv_fwd(x, w, k, k, (s, s), (p, p), stats=st, stats_part=True, cfg=cfg)
    pr = F.conv2d(xr.detach(), wr.detach(), None, stride=s, padding=p)
    tot = st.view(G, 2 * Co).sum(0)
    assert _rel(tot[:Co], pr.sum((0, 2, 3))) < 2e-2 and _rel(tot[Co:], (pr * pr).sum((0, 2, 3))) < 2e-2
    dy = _bf(torch.randn_like(pre))
    pre.backward(dy.float())
    dyh = dy.permute(0, 2, 3, 1).contiguous()
    add = _bf(torch.randn(B, H, W, Ci, device=dev))
    dx = K.conv_dgrad(dyh, w, x.shape, k, k, (s, s), (p, p), addend=add, cfg=cfg)
    assert _rel(dx.permute(0, 3, 1, 2), xr.grad + add.float().permute(0, 3, 1, 2)) < 1e-2
    dw = torch.zeros(Co, k, k, Ci, device=dev)
    K.conv_wgrad(x, dyh, dw, k, k, (s, s), (p, p), cfg=cfg)
    assert _rel(dw.permute(0, 3, 1, 2), wr.grad) < 1e-2


def test_linear_paths_match_torch():
    """Linear on the MFMA GEMM kernel: forward, input gradient, and the weight gradient
    accumulating into the fp32 gradient storage (checked by a second backward doubling the
    gradient), against fp32 torch."""
    from kubeml_amd.nn import flatten_module
    from kubeml_amd.nn import modules as Mo
    torch.manual_seed(3)
    ref = torch.nn.Linear(768, 1000).to(dev)
    lin = Mo.Linear(768, 1000).to(dev)
    lin.load_state_dict(ref.state_dict())
    flatten_module(lin)
    x = _bf(torch.randn(4096, 768, device=dev)).requires_grad_(True)
    y = lin(x)
    xr = x.detach().float().requires_grad_(True)
    yr = ref(xr)
    assert _rel(y.float(), yr) < 1e-2
    g = _bf(torch.randn_like(yr))
    y.backward(g)
    yr.backward(g.float())
    assert _rel(x.grad.float(), xr.grad) < 1e-2
    assert _rel(lin.weight.grad, ref.weight.grad) < 1e-2
    assert _rel(lin.bias.grad, ref.bias.grad) < 1e-2
    lin(x.detach()).backward(g)
    assert _rel(lin.weight.grad, 2 * ref.weight.grad) < 1e-2


@pytest.mark.parametrize("M,C", [(16384, 3072), (1000, 768), (300, 36), (100, 1000)])
def test_colsum_and_slab_sum(M, C):
    """Bias-gradient column sums (16-byte vectorised kernel when C % 8 == 0 and M >= 256,
    scalar otherwise; both accumulate) and the split-K slab fold dst += sum_s part[s]."""
    from kubeml_amd.ops import kernels as K
    torch.manual_seed(5)
    x = _bf(torch.randn(M, C, device=dev))
    out = torch.ones(C, device=dev)
    K.colsum_(x, out)
    ref = x.float().sum(0) + 1
    assert (out - ref).abs().max().item() < 1e-3 * max(1.0, ref.abs().max().item()) + 1e-2
    part = torch.randn(4, C, 8, device=dev)
    dst = torch.randn(C, 8, device=dev)
    want = dst + part.sum(0)
    K.slab_sum_add_(part, dst)
    assert torch.allclose(dst, want, atol=1e-5)


# ---------------------------------------------------------------------------------------
# unrolled 2x2-map convs (3x3 / s1 / p1 run as their dense 1x1 form, ops.kernels.unrolled22)
# ---------------------------------------------------------------------------------------

@pytest.mark.parametrize("B,C,Kc", [(256, 256, 256), (37, 64, 128), (8, 32, 24)])
def test_unrolled_conv_fwd_bn_matches_3x3(B, C, Kc):
    from kubeml_amd.ops import kernels as K
    torch.manual_seed(0)
    x = _bf(torch.randn(B, 2, 2, C, device=dev))
    w = _bf(torch.randn(Kc, 3, 3, C, device=dev) * 0.05)
    wu = K.unrolled_weight(w)
    torch.testing.assert_close(wu, K.unroll22_reference(w), rtol=0, atol=0)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    args = (3, 3, (1, 1), (1, 1))
    G3 = K.conv_fwd_stats_rows(x.shape, Kc, *args)
    Gu = K.conv_fwd_stats_rows(x.shape, Kc, *args, unroll=True)
    s3 = torch.empty(G3 * 2 * Kc, device=dev)
    su = torch.empty(Gu * 2 * Kc, device=dev)
    y3 = K.conv_fwd(x, w, *args, stats=s3, stats_part=True)
    yu = K.conv_fwd(x, w, *args, stats=su, stats_part=True, wu=wu)
    assert yu.shape == (B, 2, 2, Kc)
    assert _rel(yu, ref) < 1e-2 and _rel(y3, ref) < 1e-2
    # folded partial rows: ordinary [sum | sumsq] rows of the Kc channels (from the fp32
    # conv values, like the 3x3 path's rows: compare the two)
    tot = su.view(Gu, 2, Kc).sum(0)
    tot3 = s3.view(G3, 2, Kc).sum(0)
    torch.testing.assert_close(tot, tot3, rtol=1e-3, atol=5e-2)
    yf = yu.float().reshape(-1, Kc)
    assert _rel(tot[1], (yf * yf).sum(0)) < 1e-2
    gamma = torch.rand(Kc, device=dev) + 0.5
    beta = torch.randn(Kc, device=dev) * 0.1
    a3 = K.bn_apply(y3, s3, gamma, beta, relu=True, stats_rows=G3)
    au = K.bn_apply(yu, su, gamma, beta, relu=True, stats_rows=Gu)
    assert _rel(au, a3) < 2e-2


@pytest.mark.parametrize("B,C,Kc", [(256, 256, 256), (37, 64, 128)])
def test_unrolled_conv_bwd_matches_3x3(B, C, Kc):
    from kubeml_amd.ops import kernels as K
    torch.manual_seed(1)
    x = _bf(torch.randn(B, 2, 2, C, device=dev))
    w = _bf(torch.randn(Kc, 3, 3, C, device=dev) * 0.05)
    dy = _bf(torch.randn(B, 2, 2, Kc, device=dev))
    addend = _bf(torch.randn(B, 2, 2, C, device=dev))
    wu = K.unrolled_weight(w)
    args = (3, 3, (1, 1), (1, 1))
    xr = x.float().permute(0, 3, 1, 2).requires_grad_()
    wr = w.float().permute(0, 3, 1, 2).requires_grad_()
    (F.conv2d(xr, wr, padding=1) * dy.float().permute(0, 3, 1, 2)).sum().backward()
    dx_ref = xr.grad.permute(0, 2, 3, 1) + addend.float()
    dw_ref = wr.grad.permute(0, 2, 3, 1)
    # consumer BN of dx (channels C): its dgamma/dbeta partial rows come out folded
    yc = _bf(torch.randn(B, 2, 2, C, device=dev))
    cc = _bf(torch.randn(B, 2, 2, C, device=dev))
    mean = torch.randn(C, device=dev) * 0.1
    rstd = torch.rand(C, device=dev) + 0.5
    # weight gradient: the dense 1x1 form into a [4K,1,1,4C] scratch, folded onto the 3x3
    # taps by fold22_multi (fixed pair order: stored, or added onto what dw holds)
    g = torch.full((4 * Kc, 1, 1, 4 * C), float("nan"), device=dev)   # every element written
    dx, (part, G) = K.conv_bwd(dy, w, x, g, *args, addend=addend, bnf=(yc, cc, mean, rstd), wu=wu)
    assert dx.shape == (B, 2, 2, C)
    assert _rel(dx, dx_ref) < 1e-2
    dw = torch.full((Kc, 3, 3, C), float("nan"), device=dev)
    K.fold22_multi([(g, dw, False)])
    assert _rel(dw, dw_ref) < 1e-2
    dw_acc = torch.ones(Kc, 3, 3, C, device=dev)
    K.fold22_multi([(g, dw_acc, True)])
    torch.testing.assert_close(dw_acc, dw + 1.0, rtol=0, atol=1e-5)
    g2 = torch.empty_like(g)
    K.conv_bwd(dy, w, x, g2, *args, addend=addend, bnf=(yc, cc, mean, rstd), wu=wu)
    assert torch.equal(g, g2)                                           # deterministic
    dz = dx.float() * (yc.float() > 0)
    xh = (cc.float() - mean) * rstd
    tot = part.view(G, 2, C).sum(0)
    torch.testing.assert_close(tot[0], dz.reshape(-1, C).sum(0), rtol=2e-3, atol=2e-1)
    torch.testing.assert_close(tot[1], (dz * xh).reshape(-1, C).sum(0), rtol=2e-3, atol=2e-1)
    # the separate dgrad / wgrad entry points
    g3 = torch.empty_like(g)
    K.conv_wgrad(x, dy, g3, *args, unroll=True)
    dw2 = torch.empty_like(dw)
    K.fold22_multi([(g3, dw2, False)])
    assert torch.equal(dw2, dw)
    dx2 = K.conv_dgrad(dy, w, x.shape, *args, addend=addend, wu=wu)
    assert _rel(dx2, dx_ref) < 1e-2


@pytest.mark.parametrize("B,H,C", [(16, 16, 64), (3, 112, 64), (5, 9, 24)])
def test_bn_relu_maxpool_matches_unfused(B, H, C):
    """Fused stem BN -> ReLU -> max-pool (one pass, normalised map never written) against
    bn_apply + maxpool_fwd, and its backward (ReLU mask folded into the gather max-pool
    backward) against maxpool_bwd * [y > 0]; batch statistics from conv-style partial rows."""
    from kubeml_amd.ops import kernels as K
    torch.manual_seed(5)
    c = _bf(torch.randn(B, H, H, C, device=dev) * 2 + 0.3)
    cf = c.float().reshape(-1, C)
    G = 7
    rows = torch.zeros(G, 2, C, device=dev)
    for g, chunk in enumerate(cf.chunk(G)):
        rows[g, 0] = chunk.sum(0)
        rows[g, 1] = (chunk * chunk).sum(0)
    gamma = torch.rand(C, device=dev) + 0.5
    beta = torch.randn(C, device=dev) * 0.2
    rm1, rv1 = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    rm2, rv2 = rm1.clone(), rv1.clone()
    m1, r1 = torch.empty(C, device=dev), torch.empty(C, device=dev)
    m2, r2 = torch.empty(C, device=dev), torch.empty(C, device=dev)
    y = K.bn_apply(c, rows.reshape(-1), gamma, beta, save_mean=m1, save_rstd=r1, run_mean=rm1, run_var=rv1,
                   relu=True, stats_rows=G)
    p_ref, idx_ref = K.maxpool_fwd(y, 3, 2, 1)
    p, idx = K.bn_relu_maxpool(c, rows.reshape(-1), gamma, beta, 3, 2, 1, save_mean=m2, save_rstd=r2, run_mean=rm2,
                               run_var=rv2, stats_rows=G)
    assert p.shape == p_ref.shape
    # same statistics; values can differ by one bf16 rounding step where the two kernels'
    # FMA orders differ, which may flip an argmax between near-equal window elements
    for a, b in ((m2, m1), (r2, r1), (rm2, rm1), (rv2, rv1)):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(p.float(), p_ref.float(), rtol=1e-2, atol=1e-2)
    assert (idx == idx_ref).float().mean() > 0.995
    # exact-semantics check against fp32 torch
    ref = F.max_pool2d(torch.relu((c.float() - m1) * r1 * gamma + beta).permute(0, 3, 1, 2), 3, 2, 1)
    assert _rel(p.permute(0, 3, 1, 2), ref) < 1e-2
    dp = _bf(torch.randn_like(p.float()))
    dz = K.maxpool_bwd(dp, idx, c.shape, 3, 2, 1, relu_out=p)
    dz_ref = K.maxpool_bwd(dp, idx, c.shape, 3, 2, 1).float() * (y.float() > 0)
    agree = (dz.float() - dz_ref).abs() <= 1e-6
    assert agree.float().mean() > 0.995


@pytest.mark.parametrize("B,C,ld", [(256, 1000, 1000), (37, 10, 16), (130, 1000, 1008), (600, 1000, 1000)])
def test_ce_bwd_adds_bias_gradient(B, C, ld):
    """ce_bwd(dbias=...): same dlogits, and dbias += column sums of dlogits (the logits
    Linear's bias gradient, which that Linear then skips)."""
    from kubeml_amd.ops import kernels as K
    torch.manual_seed(8)
    logits = _bf(torch.randn(B, ld, device=dev) * 3)
    labels = torch.randint(0, C, (B,), device=dev)
    labels[3] = -100
    out3, ws, lab = K.ce_fwd(logits, labels, -100, classes=C)
    d0 = K.ce_bwd(logits, lab, ws, out3, classes=C)
    db = torch.full((ld,), 0.25, device=dev)
    d1 = K.ce_bwd(logits, lab, ws, out3, classes=C, dbias=db)
    torch.testing.assert_close(d1, d0, rtol=0, atol=0)
    want = torch.full((ld,), 0.25, device=dev)
    want[:C] += d0.float()[:, :C].sum(0)
    torch.testing.assert_close(db, want, rtol=1e-5, atol=1e-6)
    # overwrite mode (no zeroed buffer needed) and bitwise reproducibility (ordered rows)
    db2 = torch.full((ld,), float("nan"), device=dev)
    K.ce_bwd(logits, lab, ws, out3, classes=C, dbias=db2, accumulate=False)
    torch.testing.assert_close(db2[:C], d0.float()[:, :C].sum(0), rtol=1e-5, atol=1e-6)
    db3 = torch.empty_like(db2)
    K.ce_bwd(logits, lab, ws, out3, classes=C, dbias=db3, accumulate=False)
    assert torch.equal(db2[:C], db3[:C])


@pytest.mark.parametrize("B,C,K,grouped", [(256, 512, 1000, True), (256, 512, 1000, False), (96, 64, 24, True)])
def test_wgrad_ones_column_bias_gradient(B, C, K, grouped):
    """conv_wgrad / conv_bwd(dbias=...) of a Linear (1x1 conv on a 1x1 map): the bias
    gradient comes out of the wgrad GEMM's extra ones column; dW is unchanged by it."""
    from kubeml_amd.ops import kernels as K_
    torch.manual_seed(11)
    x = _bf(torch.randn(B, 1, 1, C, device=dev))
    dy = _bf(torch.randn(B, 1, 1, K, device=dev))
    w = _bf(torch.randn(K, 1, 1, C, device=dev) * 0.05)
    want_db = dy.float().reshape(B, K).sum(0)
    want_dw = (dy.float().reshape(B, K).t() @ x.float().reshape(B, C)).reshape(K, 1, 1, C)
    dw = torch.full((K, 1, 1, C), float("nan"), device=dev)
    db = torch.full((K,), float("nan"), device=dev)
    if grouped:
        dx = K_.conv_bwd(dy, w, x, dw, 1, 1, (1, 1), (0, 0), accumulate=False, dbias=db, bias_accumulate=False)
        torch.testing.assert_close(dx.float().reshape(B, C), dy.float().reshape(B, K) @ w.float().reshape(K, C),
                                   rtol=2e-2, atol=2e-2)
    else:
        K_.conv_wgrad(x, dy, dw, 1, 1, (1, 1), (0, 0), accumulate=False, dbias=db, bias_accumulate=False)
    torch.testing.assert_close(db, want_db, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(dw, want_dw, rtol=1e-5, atol=1e-4)
    # accumulate mode adds
    db2 = torch.full((K,), 0.5, device=dev)
    dw2 = torch.zeros_like(dw)
    K_.conv_wgrad(x, dy, dw2, 1, 1, (1, 1), (0, 0), accumulate=True, dbias=db2, bias_accumulate=True)
    torch.testing.assert_close(db2, want_db + 0.5, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("B,C,Kc", [(64, 256, 256), (32, 128, 256), (8, 64, 32)])
def test_gathered_unrolled_weight_matches_materialised(B, C, Kc):
    """wu=GATHER22: the FWD / DGRAD loaders gather the unrolled weight straight from the 3x3
    weight — bitwise the same results as the materialised [4K,1,1,4C] copy, for the forward
    (with folded BN partial rows), the dgrad and the grouped dgrad+wgrad launch."""
    from kubeml_amd.ops import kernels as K
    torch.manual_seed(3)
    x = _bf(torch.randn(B, 2, 2, C, device=dev))
    w = _bf(torch.randn(Kc, 3, 3, C, device=dev) * 0.05)
    dy = _bf(torch.randn(B, 2, 2, Kc, device=dev))
    wu = K.unrolled_weight(w)
    args = (3, 3, (1, 1), (1, 1))
    Gu = K.conv_fwd_stats_rows(x.shape, Kc, *args, unroll=True)
    s1 = torch.empty(Gu * 2 * Kc, device=dev)
    s2 = torch.empty(Gu * 2 * Kc, device=dev)
    y1 = K.conv_fwd(x, w, *args, stats=s1, stats_part=True, wu=wu)
    y2 = K.conv_fwd(x, w, *args, stats=s2, stats_part=True, wu=K.GATHER22)
    assert torch.equal(y1, y2) and torch.equal(s1, s2)
    plan = K.bwd_plans(x.shape, Kc, *args, unroll=True)[0]
    if plan[4] != K.DIRECT:
        d1 = K.conv_dgrad(dy, w, x.shape, *args, wu=wu)
        d2 = K.conv_dgrad(dy, w, x.shape, *args, wu=K.GATHER22)
        assert torch.equal(d1, d2)
        g1 = torch.empty((4 * Kc, 1, 1, 4 * C), device=dev)
        g2 = torch.empty_like(g1)
        e1 = K.conv_bwd(dy, w, x, g1, *args, wu=wu)
        e2 = K.conv_bwd(dy, w, x, g2, *args, wu=K.GATHER22)
        assert torch.equal(e1, e2) and torch.equal(g1, g2)


@pytest.mark.parametrize("shape", [(40, 1, 1, 512, 512, 3, 1, 1), (37, 1, 1, 512, 96, 1, 1, 0),
                                   (30, 2, 2, 256, 256, 1, 1, 0), (33, 1, 1, 256, 64, 1, 1, 0)])
def test_conv_oneshot_variant(shape):
    """One-shot panel forward (variant 5, LDS-DMA of the whole K panels): single-tap convs
    (centre tap on 1x1 maps, 1x1/s1) vs fp32 torch, with bias/ReLU/atomic statistics and the
    per-M-tile partial rows; M and N tails included."""
    from kubeml_amd.ops import kernels as K
    B, H, W, Ci, Co, k, s, p = shape
    torch.manual_seed(13)
    x = _bf(torch.randn(B, H, W, Ci, device=dev))
    w = _bf(torch.randn(Co, k, k, Ci, device=dev) * (1.0 / Ci ** 0.5))
    bias = torch.randn(Co, device=dev)
    pre = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), bias, stride=s, padding=p)
    tiles = [t for t in K._ONESHOT_TILES[Ci]]
    assert K.oneshot_plan(Ci, Co, Ci, H, W, k, k, (s, s), (p, p)) is not None
    for bm, bn in tiles:
        cfg = (bm, bn, 0, 1, K.ONESHOT)
        st = torch.zeros(2 * Co, device=dev)
        y = K.conv_fwd(x, w, k, k, (s, s), (p, p), bias=bias, stats=st, relu=True, cfg=cfg)
        yr = F.relu(pre)
        assert _rel(y.permute(0, 3, 1, 2), yr) < 1e-2, (bm, bn)
        assert _rel(st[:Co], yr.sum((0, 2, 3))) < 2e-2, (bm, bn)
        G = K.conv_fwd_stats_rows(x.shape, Co, k, k, (s, s), (p, p), cfg=cfg)
        buf = torch.full((G * 2 * Co + 256,), float("nan"), device=dev)
        y2 = K.conv_fwd(x, w, k, k, (s, s), (p, p), stats=buf[:G * 2 * Co], stats_part=True, cfg=cfg)
        assert torch.isnan(buf[G * 2 * Co:]).all() and not torch.isnan(buf[:G * 2 * Co]).any()
        yf = pre - bias.view(1, -1, 1, 1)
        assert _rel(y2.permute(0, 3, 1, 2), yf) < 1e-2
        assert _rel(buf[:G * 2 * Co].view(G, 2, Co).sum(0)[0], yf.sum((0, 2, 3))) < 2e-2


def test_conv_oneshot_unrolled_gather():
    """Unrolled 2x2-map conv (1x1 form, K = 4C = 1024) on the one-shot kernel with the B rows
    gathered from the 3x3 weight (GATHER22): equals the 3x3 conv, folded statistics included."""
    from kubeml_amd.ops import kernels as K
    torch.manual_seed(14)
    B, C, Co = 24, 256, 256
    x = _bf(torch.randn(B, 2, 2, C, device=dev))
    w = _bf(torch.randn(Co, 3, 3, C, device=dev) * (1.0 / (9 * C) ** 0.5))
    args = (3, 3, (1, 1), (1, 1))
    assert K.conv_fwd_plan(4 * C, B, 4 * Co, 4 * C, geom=(1, 1, 1, 1, (1, 1), (0, 0)))[4] == K.ONESHOT
    G = K.conv_fwd_stats_rows(x.shape, Co, *args, unroll=True)
    st = torch.empty(G * 2 * Co, device=dev)
    y = K.conv_fwd(x, w, *args, stats=st, stats_part=True, wu=K.GATHER22)
    yr = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), padding=1)
    assert _rel(y.permute(0, 3, 1, 2), yr) < 1e-2
    rows = st.view(G, 2, Co).sum(0)
    assert _rel(rows[0], yr.sum((0, 2, 3))) < 2e-2 and _rel(rows[1], (yr * yr).sum((0, 2, 3))) < 2e-2


@pytest.mark.parametrize("unroll", [False, True])
def test_conv_oneshot_backward(unroll, monkeypatch):
    """One-shot dgrad / wgrad bodies (K-strided panels by LDS-DMA, transposing reads) on the
    batch-256 single-tap convs they are planned for: layer4's centre-tap 3x3 on 1x1 maps and
    layer3's unrolled 2x2 convs (1x1 form, gathered weight, folded BN partials) vs fp32 torch."""
    from kubeml_amd.ops import kernels as K
    monkeypatch.setattr(K, "_ONESHOT_BWD_ON", True)     # opt-in in the step
    torch.manual_seed(15)
    B, H, C, Co = (256, 2, 256, 256) if unroll else (256, 1, 512, 512)
    x = _bf(torch.randn(B, H, H, C, device=dev))
    w = _bf(torch.randn(Co, 3, 3, C, device=dev) * (1.0 / (9 * C) ** 0.5))
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.conv2d(xr, wr, padding=1)
    dy = _bf(torch.randn_like(yr))
    yr.backward(dy.float())
    dyn = dy.permute(0, 2, 3, 1).contiguous()
    add = _bf(torch.randn(B, H, H, C, device=dev))
    dplan, wplan, _ = K.bwd_plans(x.shape, Co, 3, 3, (1, 1), (1, 1), unroll=unroll)
    assert dplan[4] == K.ONESHOT and wplan[4] == K.ONESHOT
    if unroll:
        dw = torch.full((4 * Co, 1, 1, 4 * C), float("nan"), device=dev)
        dx = K.conv_bwd(dyn, w, x, dw, 3, 3, (1, 1), (1, 1), addend=add, wu=K.GATHER22)
        dw3 = torch.zeros(Co, 3, 3, C, device=dev)
        K.fold22_multi([(dw, dw3, False)])
    else:
        dw3 = torch.full((Co, 3, 3, C), float("nan"), device=dev)
        dx = K.conv_bwd(dyn, w, x, dw3, 3, 3, (1, 1), (1, 1), addend=add, accumulate=False)
        # on a 1x1 map only the centre tap has a gradient (the others see padding only)
        dw3 = dw3[:, 1:2, 1:2, :]
    gref = wr.grad if unroll else wr.grad[:, :, 1:2, 1:2]
    assert _rel(dx.permute(0, 3, 1, 2), xr.grad + add.float().permute(0, 3, 1, 2)) < 1e-2
    assert _rel(dw3.permute(0, 3, 1, 2), gref) < 1e-2


def test_conv_stem_variant():
    """Stem halo kernel (variant 6: 7x7/s2/p3 on a 32x32 image, Cin 3 padded to 8, one image per
    block) vs fp32 torch: output, atomic statistics and one partial row per image."""
    from kubeml_amd.ops import kernels as K
    torch.manual_seed(16)
    B = 5
    x = torch.zeros(B, 32, 32, 8, device=dev)
    x[..., :3] = torch.randn(B, 32, 32, 3, device=dev)
    x = _bf(x)
    w = torch.zeros(64, 7, 7, 8, device=dev)
    w[..., :3] = torch.randn(64, 7, 7, 3, device=dev) * 0.1
    w = _bf(w)
    cfg = K.conv_fwd_plan(8, B * 256, 64, 392, geom=(32, 32, 7, 7, (2, 2), (3, 3)))
    assert cfg[4] == K.STEM
    yr = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), stride=2, padding=3)
    st = torch.zeros(128, device=dev)
    y = K.conv_fwd(x, w, 7, 7, (2, 2), (3, 3), stats=st, cfg=cfg)
    assert _rel(y.permute(0, 3, 1, 2), yr) < 1e-2
    assert _rel(st[:64], yr.sum((0, 2, 3))) < 2e-2 and _rel(st[64:], (yr * yr).sum((0, 2, 3))) < 2e-2
    G = K.conv_fwd_stats_rows(x.shape, 64, 7, 7, (2, 2), (3, 3))
    assert G == B
    buf = torch.full((G * 128 + 64,), float("nan"), device=dev)
    y2 = K.conv_fwd(x, w, 7, 7, (2, 2), (3, 3), stats=buf[:G * 128], stats_part=True)
    assert torch.equal(y, y2) and torch.isnan(buf[G * 128:]).all()
    assert _rel(buf[:G * 128].view(G, 2, 64).sum(0)[0], yr.sum((0, 2, 3))) < 2e-2


@pytest.mark.parametrize("B", [3, 300])
def test_conv_stem_rows_224(B):
    """ImageNet-size stem (variant 6 on 224x224: persistent blocks over output row pairs,
    weights resident in LDS) vs fp32 torch: output and one partial statistics row per row
    pair.  B = 300 has more tiles (16800) than blocks, so blocks loop and prefetch."""
    from kubeml_amd.ops import kernels as K
    torch.manual_seed(18)
    x = torch.zeros(B, 224, 224, 8, device=dev)
    x[..., :3] = torch.randn(B, 224, 224, 3, device=dev)
    x = _bf(x)
    w = torch.zeros(64, 7, 7, 8, device=dev)
    w[..., :3] = torch.randn(64, 7, 7, 3, device=dev) * 0.1
    w = _bf(w)
    M = B * 112 * 112
    cfg = K.conv_fwd_plan(8, M, 64, 392, geom=(224, 224, 7, 7, (2, 2), (3, 3)))
    assert cfg[4] == K.STEM and cfg[0] == 224
    G = K.conv_fwd_stats_rows(x.shape, 64, 7, 7, (2, 2), (3, 3))
    assert G == B * 56
    buf = torch.full((G * 128 + 64,), float("nan"), device=dev)
    y = K.conv_fwd(x, w, 7, 7, (2, 2), (3, 3), stats=buf[:G * 128], stats_part=True)
    torch.cuda.synchronize()
    assert torch.isnan(buf[G * 128:]).all() and not torch.isnan(buf[:G * 128]).any()
    for b0 in sorted({0, B // 2, B - 1}):
        yr = F.conv2d(x[b0:b0 + 1].float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), stride=2, padding=3)
        assert _rel(y[b0:b0 + 1].permute(0, 3, 1, 2), yr) < 1e-2
        rows = buf[:G * 128].view(B, 56, 2, 64)[b0]
        assert _rel(rows[:, 0].sum(0), yr.sum((0, 2, 3))) < 2e-2
        assert _rel(rows[:, 1].sum(0), (yr * yr).sum((0, 2, 3))) < 2e-2
        # one row per output row pair: row t covers output rows 2t, 2t+1
        assert _rel(rows[7, 0], yr[0, :, 14:16].sum((1, 2))) < 2e-2


@pytest.mark.parametrize("case", [(8, 8, 64, 64), (12, 4, 128, 128)])
def test_conv_fwd_bnin_matches_bn_then_conv(case):
    """conv_fwd_bnin (the input's BN + ReLU applied while the halo patch is staged) vs
    bn_apply followed by the halo conv: normalised input, saved statistics, running buffers
    and the conv output (+ its partial rows); the producer's rows group-reduced or not."""
    from kubeml_amd.ops import kernels as K
    B, H, C, Co = case
    torch.manual_seed(17)
    x = _bf(torch.randn(B, H, H, C, device=dev))
    w1 = _bf(torch.randn(C, 3, 3, C, device=dev) * (1.0 / (9 * C) ** 0.5))
    w2 = _bf(torch.randn(Co, 3, 3, C, device=dev) * (1.0 / (9 * C) ** 0.5))
    g, b = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    for group in (False, True):
        G1 = K.conv_fwd_stats_rows(x.shape, C, 3, 3, (1, 1), (1, 1), group=group)
        rows = torch.empty(G1 * 2 * C, device=dev)
        c1 = K.conv_fwd(x, w1, 3, 3, (1, 1), (1, 1), stats=rows, stats_part=True, stats_group=group)
        # reference: BN apply kernel, then the conv
        m0, r0 = torch.empty(C, device=dev), torch.empty(C, device=dev)
        rm0, rv0 = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        y0 = K.bn_apply(c1, rows, g, b, save_mean=m0, save_rstd=r0, run_mean=rm0, run_var=rv0, relu=True,
                        stats_rows=G1)
        o0 = K.conv_fwd(y0, w2, 3, 3, (1, 1), (1, 1))
        # folded
        m1, r1 = torch.empty(C, device=dev), torch.empty(C, device=dev)
        rm1, rv1 = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        y1 = torch.full_like(c1, float("nan"))
        G2 = K.conv_fwd_stats_rows(c1.shape, Co, 3, 3, (1, 1), (1, 1))
        st2 = torch.empty(G2 * 2 * Co, device=dev)
        o1 = K.conv_fwd_bnin(c1, w2, rows, G1, g, b, m1, r1, rm1, rv1, 1e-5, 0.1, y1, stats=st2)
        torch.testing.assert_close(m1, m0, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(r1, r0, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(rm1, rm0, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(rv1, rv0, rtol=1e-5, atol=1e-6)
        assert not torch.isnan(y1.float()).any(), group
        assert _rel(y1, y0) < 1e-2, (group, _rel(y1, y0))
        if not group:   # same rows, same summation order and arithmetic as the BN apply kernel
            assert torch.equal(y1, y0) and torch.equal(m1, m0) and torch.equal(r1, r0)
        assert _rel(o1, o0) < 1e-2, (group, _rel(o1, o0))
        of = o1.float().reshape(-1, Co)
        assert _rel(st2.view(G2, 2, Co).sum(0)[0], of.sum(0)) < 2e-2


@pytest.mark.parametrize("shape", [(8, 56, 56, 64, 64, 3, 1), (8, 57, 57, 64, 128, 3, 1), (8, 56, 56, 128, 64, 1, 0),
                                   (8, 57, 56, 64, 64, 1, 0)])
@pytest.mark.parametrize("cfg", [(64, 64, 32, 1, 0), (64, 64, 64, 1, 0), (64, 128, 64, 1, 1)])
def test_stride2_dgrad_parity_classes(shape, cfg, monkeypatch):
    """Stride-2 dgrad as four parity-class launches == the plain stride-2 dgrad (bit-exact dX,
    same consumer-BN dgamma/dbeta) and the fp32 torch reference; with and without addend."""
    from kubeml_amd.ops import kernels as K
    B, H, W, Ci, Co, k, p = shape
    assert K.s2_parity_ok(B, H, W, (2, 2), cfg)
    torch.manual_seed(11)
    OH, OW = K.out_hw(H, W, k, k, 2, 2, p, p)
    dy = _bf(torch.randn(B, OH, OW, Co, device=dev))
    w = _bf(torch.randn(Co, k, k, Ci, device=dev) * 0.05)
    add = _bf(torch.randn(B, H, W, Ci, device=dev))
    c = _bf(torch.randn(B, H, W, Ci, device=dev))
    ybn = _bf(torch.randn(B, H, W, Ci, device=dev))
    mean, rstd = torch.randn(Ci, device=dev), torch.rand(Ci, device=dev) + 0.5
    g = torch.rand(Ci, device=dev) + 0.5
    for addend in (add, None):
        for mask in (False, True):
            dx1, part1 = K.conv_dgrad(dy, w, (B, H, W, Ci), k, k, (2, 2), (p, p), addend=addend, cfg=cfg,
                                      bnf=(ybn, c, mean, rstd), bnf_mask=mask)
            monkeypatch.setattr(K, "_S2_PARITY_MIN_ROWS", 1 << 40)
            dx0, part0 = K.conv_dgrad(dy, w, (B, H, W, Ci), k, k, (2, 2), (p, p), addend=addend, cfg=cfg,
                                      bnf=(ybn, c, mean, rstd), bnf_mask=mask)
            monkeypatch.setattr(K, "_S2_PARITY_MIN_ROWS", 20000)
            torch.cuda.synchronize()
            assert torch.equal(dx1, dx0)
            dg0, db0 = torch.zeros(Ci, device=dev), torch.zeros(Ci, device=dev)
            dg1, db1 = torch.zeros(Ci, device=dev), torch.zeros(Ci, device=dev)
            yy = None if mask else ybn
            K.bn_bwd(dx0, yy, c, mean, rstd, g, dg0, db0, partial=part0)
            K.bn_bwd(dx1, yy, c, mean, rstd, g, dg1, db1, partial=part1)
            assert _rel(db1, db0) < 1e-4 and _rel(dg1, dg0) < 1e-4
    xr = torch.zeros(B, Ci, H, W, device=dev, requires_grad=True)
    F.conv2d(xr, w.float().permute(0, 3, 1, 2), stride=2, padding=p).backward(dy.float().permute(0, 3, 1, 2))
    dx = K.conv_dgrad(dy, w, (B, H, W, Ci), k, k, (2, 2), (p, p), cfg=cfg)
    assert _rel(dx, xr.grad.permute(0, 2, 3, 1)) < 1e-2


@pytest.mark.parametrize("n,n_params", [(4099, 4096), (1 << 20, (1 << 20) - 40)])
def test_kavg_async_snap_and_apply_match_torch(n, n_params):
    """Fused staleness-1 K-AVG passes == the torch ops they replace, bit for bit: the flat /
    snap copies, x + (flat / world - snap) (torch divides by a scalar as a multiply by the
    fp32 reciprocal; the kernel keeps that product rounded on its own, no FMA), and the
    shadow is bf16(x) over the parameters."""
    from kubeml_amd.ops import kernels as K
    torch.manual_seed(19)
    x = torch.randn(n, device=dev)
    flat, snap = torch.empty_like(x), torch.empty_like(x)
    K.kavg_snap_(x, flat, snap)
    assert torch.equal(flat, x) and torch.equal(snap, x)
    flat.mul_(3.0).add_(torch.randn_like(x))          # the "all-reduced" sum
    x2 = x + torch.randn_like(x) * 0.01                # local progress since the snapshot
    ref = x2.clone()
    ref.add_(flat.clone().div_(3).sub_(snap))
    shadow = torch.zeros(n_params, dtype=torch.bfloat16, device=dev)
    K.kavg_async_apply_(x2, flat, snap, shadow, 3, n_params)
    torch.cuda.synchronize()
    assert torch.equal(x2, ref), int((x2 != ref).sum())
    assert torch.equal(shadow, ref[:n_params].to(torch.bfloat16))


@pytest.mark.parametrize("route", [("slab", 128, 128, 2, 16), ("slab", 128, 128, 2, 4)])
def test_conv1x1_wgrad_gemm_routes(monkeypatch, route):
    """1x1/s1 conv weight gradient on a GEMM route (wgrad_gemm.json): the slab split-K kernel
    (hand-written; no library route is left), stored and accumulated, alone and through conv_bwd (which then runs the
    dgrad on its own) — against fp32 torch."""
    from kubeml_amd.ops import kernels as K
    torch.manual_seed(23)
    B, H, W, C, Co = 8, 14, 14, 64, 128
    monkeypatch.setitem(K._WGRAD_GEMM, (B * H * W, Co, C), route)
    x = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
    dy = torch.randn(B, H, W, Co, device=dev).to(torch.bfloat16)
    w = (torch.randn(Co, 1, 1, C, device=dev) * 0.05).to(torch.bfloat16)
    ref = (dy.reshape(-1, Co).double().t() @ x.reshape(-1, C).double()).view(Co, 1, 1, C)
    dw = torch.full((Co, 1, 1, C), 7.0, device=dev)
    K.conv_wgrad(x, dy, dw, 1, 1, (1, 1), (0, 0), accumulate=False)
    assert _rel(dw, ref) < 1e-5
    K.conv_wgrad(x, dy, dw, 1, 1, (1, 1), (0, 0), accumulate=True)
    assert _rel(dw, 2 * ref) < 1e-5
    dw2 = torch.zeros_like(dw)
    dx = K.conv_bwd(dy, w, x, dw2, 1, 1, (1, 1), (0, 0))
    assert _rel(dw2, ref) < 1e-5
    assert _rel(dx, dy.float() @ w.view(Co, C).float()) < 1e-2
