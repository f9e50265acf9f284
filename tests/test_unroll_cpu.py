"""The unrolled form of a 3x3 / stride 1 / pad 1 conv on a 2x2 map (ops.kernels.unrolled22)
is exact: forward, input gradient and weight gradient (scatter back onto the taps) equal
the 3x3 conv's.  Checks the index mapping the HIP kernels use, in fp64 on the CPU."""
import torch
import torch.nn.functional as F

from kubeml_amd.ops import kernels as K


def _setup(B=3, C=8, Kc=16, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, 2, 2, C, generator=g, dtype=torch.float64)          # NHWC
    w = torch.randn(Kc, 3, 3, C, generator=g, dtype=torch.float64)         # KRSC
    return x, w


def _conv_nhwc(x, w):
    y = F.conv2d(x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), padding=1)
    return y.permute(0, 2, 3, 1)


def test_unrolled_forward_is_the_3x3_conv():
    x, w = _setup()
    B, _, _, C = x.shape
    Kc = w.shape[0]
    wu = K.unroll22_reference(w).reshape(4 * Kc, 4 * C)
    y = (x.reshape(B, 4 * C) @ wu.t()).reshape(B, 2, 2, Kc)
    torch.testing.assert_close(y, _conv_nhwc(x, w), rtol=1e-12, atol=1e-12)


def test_unrolled_gradients_match_and_wgrad_scatter_mapping():
    x, w = _setup(seed=1)
    B, _, _, C = x.shape
    Kc = w.shape[0]
    xr, wr = x.clone().requires_grad_(), w.clone().requires_grad_()
    dy = torch.randn(B, 2, 2, Kc, dtype=torch.float64)
    (_conv_nhwc(xr, wr) * dy).sum().backward()
    wu = K.unroll22_reference(w).reshape(4 * Kc, 4 * C)
    dx = (dy.reshape(B, 4 * Kc) @ wu).reshape(B, 2, 2, C)
    torch.testing.assert_close(dx, xr.grad, rtol=1e-12, atol=1e-12)
    # wgrad of the dense form, scattered onto taps exactly as the WGRAD epilogue does
    dwu = dy.reshape(B, 4 * Kc).t() @ x.reshape(B, 4 * C)                  # [(p,n)][(q,c)]
    dw = torch.zeros(Kc, 9, C, dtype=torch.float64)
    for row in range(4 * Kc):
        p, n = divmod(row, Kc)
        for q in range(4):
            tap = ((q >> 1) - (p >> 1) + 1) * 3 + ((q & 1) - (p & 1) + 1)
            dw[n, tap] += dwu[row, q * C:(q + 1) * C]
    torch.testing.assert_close(dw.reshape(Kc, 3, 3, C), wr.grad, rtol=1e-12, atol=1e-12)


def test_unrolled_only_for_2x2_stride1_pad1_3x3():
    assert K.unrolled22(2, 2, 3, 3, (1, 1), (1, 1))
    assert not K.unrolled22(4, 4, 3, 3, (1, 1), (1, 1))
    assert not K.unrolled22(2, 2, 3, 3, (2, 2), (1, 1))
    assert not K.unrolled22(2, 2, 1, 1, (1, 1), (0, 0))
