"""Hand-written MFMA GEMM (csrc/kernels/gemm.hip) against fp32 PyTorch references: the
three linear-layer GEMMs (forward with bias / erf-GELU / pre-activation copy, dgrad,
fp32 weight-gradient accumulate and split-K atomics), every tile shape, ragged edges."""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _rand(*s, scale=1.0):
    return (torch.randn(*s, device=dev) * scale).to(torch.bfloat16)


@pytest.mark.parametrize("tile", [(256, 256), (256, 256, 4), (256, 256, 8), (256, 192, 8), (256, 128), (128, 256),
                                  (128, 128), (128, 128, 2), (128, 128, 3, "mf32"), (128, 128, 2, "mf32")])
@pytest.mark.parametrize("T,ip,op", [(512, 768, 2304), (200, 72, 136), (1216, 768, 1000)])
def test_forward_bias_gelu(tile, T, ip, op):
    from kubeml_amd.ops import gemm as G
    torch.manual_seed(0)
    x, w = _rand(T, ip), _rand(op, ip, scale=0.05)
    b = torch.randn(op, device=dev)
    y = torch.empty(T, op, dtype=torch.bfloat16, device=dev)
    pre = torch.empty_like(y)
    G.gemm(x, ip, w, ip, y, op, T, op, ip, 0, 0, bias=b, act=1, c2=pre, tile=tile, splits=1)
    h = x.float() @ w.float().t() + b
    assert _rel(pre, h) < 1e-2
    assert _rel(y, torch.nn.functional.gelu(h)) < 1e-2


@pytest.mark.parametrize("tile", [(256, 256), (256, 256, 4), (256, 256, 8), (256, 192, 8), (128, 128)])
@pytest.mark.parametrize("T,ip,op", [(512, 768, 3072), (200, 72, 136), (768, 2304, 768)])
def test_dgrad(tile, T, ip, op):
    from kubeml_amd.ops import gemm as G
    torch.manual_seed(1)
    dy, w = _rand(T, op), _rand(op, ip, scale=0.05)
    dx = torch.empty(T, ip, dtype=torch.bfloat16, device=dev)
    G.gemm(dy, op, w, ip, dx, ip, T, ip, op, 1, 0, tile=tile, splits=1)
    assert _rel(dx, dy.float() @ w.float()) < 1e-2


@pytest.mark.parametrize("tile,splits", [((256, 256), 1), ((256, 256, 4), 1), ((256, 256, 4), 2), ((256, 256, 8), 1),
                                         ((256, 256, 8), 3), ((256, 192, 8), 1), ((256, 192, 8), 3), ((128, 128), 1),
                                         ((256, 128), 4), ((128, 128), 3)])
@pytest.mark.parametrize("T,ip,op", [(2048, 768, 768), (200, 72, 136)])
def test_wgrad_accumulates(tile, splits, T, ip, op):
    from kubeml_amd.ops import gemm as G
    torch.manual_seed(2)
    dy, x = _rand(T, op), _rand(T, ip)
    dw0 = torch.randn(op, ip, device=dev)
    dw = dw0.clone()
    G.gemm(dy, op, x, ip, dw, ip, op, ip, T, 2, 2 if splits > 1 else 1, beta=1.0, tile=tile, splits=splits)
    ref = dw0.double() + dy.double().t() @ x.double()
    assert _rel(dw, ref) < 1e-4


@pytest.mark.parametrize("tile", [(256, 256, 8), (256, 192, 8)])
@pytest.mark.parametrize("layout", [0, 1, 2])
@pytest.mark.parametrize("K", [8, 64, 96, 128, 320, 4096])
def test_phase_tile_reduction_lengths(layout, K, tile):
    """k_gemm8's five-half-tiles-ahead DMA schedule and group stagger at every pipeline
    depth: a single partial K-tile up to a long reduction; ragged M / N edges."""
    from kubeml_amd.ops import gemm as G
    torch.manual_seed(5 + K)
    M, N = 296, 264
    if layout == 0:
        A, B = _rand(M, K), _rand(N, K, scale=0.05)
        C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        G.gemm(A, K, B, K, C, N, M, N, K, 0, 0, tile=tile, splits=1)
        ref = A.double() @ B.double().t()
        tol = 1e-2
    elif layout == 1:
        A, B = _rand(M, K), _rand(K, N, scale=0.05)
        C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        G.gemm(A, K, B, N, C, N, M, N, K, 1, 0, tile=tile, splits=1)
        ref = A.double() @ B.double()
        tol = 1e-2
    else:
        A, B = _rand(K, M), _rand(K, N)
        C = torch.zeros(M, N, device=dev)
        G.gemm(A, M, B, N, C, N, M, N, K, 2, 1, beta=1.0, tile=tile, splits=1)
        ref = A.double().t() @ B.double()
        tol = 1e-4
    assert _rel(C, ref) < tol


@pytest.mark.parametrize("tile,splits", [((256, 256, 8), None), ((256, 256, 8), 5), ((256, 256, 4), 3),
                                         ((128, 128, 2), 2), ((128, 128), 7)])
@pytest.mark.parametrize("T,ip,op", [(4096, 768, 2304), (1000, 72, 136)])
def test_wgrad_slab_split_k(tile, splits, T, ip, op):
    """Deterministic slab split-K weight gradient: fp32 partial tiles summed in slice order,
    bit-identical across repeated launches (no atomics)."""
    from kubeml_amd.ops import gemm as G
    torch.manual_seed(6)
    dy, x = _rand(T, op), _rand(T, ip)
    dw0 = torch.randn(op, ip, device=dev)
    dw = dw0.clone()
    G.wgrad_splitk_(dw, dy, op, x, ip, op, ip, T, beta=1.0, tile=tile, splits=splits)
    ref = dw0.double() + dy.double().t() @ x.double()
    assert _rel(dw, ref) < 1e-4
    dw2 = dw0.clone()
    G.wgrad_splitk_(dw2, dy, op, x, ip, op, ip, T, beta=1.0, tile=tile, splits=splits)
    assert torch.equal(dw, dw2)


def test_dgrad_split_k_long_reduction():
    """MLM-decoder-shaped input gradient (few output tiles, K = 30528): split-K path."""
    from kubeml_amd.ops import gemm as G
    torch.manual_seed(4)
    T, ip, op = 1216, 768, 30528
    assert G.plan(1, T, ip, op)[1] > 1
    dy, w = _rand(T, op), _rand(op, ip, scale=0.05)
    assert _rel(G.linear_dgrad(dy, w), dy.float() @ w.float()) < 1e-2


def test_linear_helpers_match_torch():
    from kubeml_amd.ops import gemm as G
    torch.manual_seed(3)
    T, ip, op = 4096, 768, 3072
    x, w = _rand(T, ip), _rand(op, ip, scale=0.05)
    b = torch.randn(op, device=dev)
    y = G.linear_fwd(x, w, b)
    assert _rel(y, x.float() @ w.float().t() + b) < 1e-2
    dy = _rand(T, op)
    assert _rel(G.linear_dgrad(dy, w), dy.float() @ w.float()) < 1e-2
    dw = torch.zeros(op, ip, device=dev)
    G.linear_wgrad_(dw, dy, x)
    assert _rel(dw, dy.double().t() @ x.double()) < 1e-4
    with pytest.raises(ValueError):
        G.linear_fwd(x, w[:, :700])


@pytest.mark.parametrize("tile", [(256, 256), (256, 256, 4), (256, 256, 8), (256, 192, 8), (256, 128), (128, 256),
                                  (128, 128), (128, 128, 2)])
@pytest.mark.parametrize("T,ip,op", [(512, 768, 2304), (200, 72, 136)])
def test_dgrad_plus_addend_equals_separate_add(tile, T, ip, op):
    """act=ADD_C2 (the transformer's residual-gradient sum fused into the dgrad epilogue):
    bit-identical to the plain dgrad followed by a bf16 add."""
    from kubeml_amd.ops import gemm as G
    torch.manual_seed(3)
    dy, w = _rand(T, op), _rand(op, ip, scale=0.05)
    add = _rand(T, ip)
    dx = torch.empty(T, ip, dtype=torch.bfloat16, device=dev)
    G.gemm(dy, op, w, ip, dx, ip, T, ip, op, 1, 0, tile=tile, splits=1)
    dx2 = torch.empty_like(dx)
    G.gemm(dy, op, w, ip, dx2, ip, T, ip, op, 1, 0, tile=tile, splits=1, c2=add, act=G.ADD_C2)
    torch.testing.assert_close(dx2, (dx.float() + add.float()).to(torch.bfloat16), rtol=0, atol=0)


def test_linear_dgrad_addend_paths():
    """linear_dgrad(addend=...) on the direct and the split-K (fp32 scratch) routes."""
    from kubeml_amd.ops import gemm as G
    torch.manual_seed(4)
    for T, ip, op in [(1024, 768, 3072), (2432, 768, 30528)]:
        dy, w = _rand(T, op), _rand(op, ip, scale=0.02)
        add = _rand(T, ip)
        ref = G.linear_dgrad(dy, w)
        want = (ref.float() + add.float()).to(torch.bfloat16)
        out = G.linear_dgrad(dy, w, addend=add)
        if G.plan(1, T, ip, op)[1] == 1:
            torch.testing.assert_close(out, want, rtol=0, atol=0)
        else:   # fp32 split-K atomics: summation order differs run to run
            assert _rel(out, want) < 1e-2



@pytest.mark.parametrize("tile", [(128, 128, 3, "mf32"), (128, 128, 2, "mf32")])
@pytest.mark.parametrize("M,N,K", [(384, 256, 512), (200, 136, 72)])
def test_mfma32_fp32_out_beta(tile, M, N, K):
    """The 32x32x16 fragment form (tiles 8 / 9) with the fp32 beta epilogue: every accumulator
    register lands on its (row, column) (a swapped row group or column half would show here)."""
    from kubeml_amd.ops import gemm as G
    torch.manual_seed(1)
    a, b = _rand(M, K), _rand(N, K)
    c0 = torch.randn(M, N, device=dev)
    c = c0.clone()
    G.gemm(a, K, b, K, c, N, M, N, K, 0, 1, beta=0.5, tile=tile, splits=1)
    assert _rel(c, 0.5 * c0 + a.float() @ b.float().t()) < 1e-5
