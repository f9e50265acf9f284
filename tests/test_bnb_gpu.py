"""BatchNorm backward folded into the conv backward pair's dz staging
(kernels.conv_bwd(bnb=...), csrc/kernels/conv_igemm.hip IgemmBody BNB) against a plain fp32
PyTorch reference of the same ops: dc = BN backward of dz, then the conv's input and weight
gradients of dc, and dgamma / dbeta."""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("B,H,C,K,G,acc", [(256, 1, 512, 512, 8, False), (64, 2, 128, 256, 40, True),
                                           (32, 4, 64, 128, 3, False)])
def test_conv_bwd_bnb_matches_fp32_reference(B, H, C, K, G, acc):
    from kubeml_amd.ops import kernels as Kk
    torch.manual_seed(B + H + C)
    x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
    w = (torch.randn(K, 3, 3, C, device=dev) * 0.05).to(torch.bfloat16)
    c = torch.randn(B, H, H, K, device=dev).to(torch.bfloat16)
    dz = torch.randn(B, H, H, K, device=dev)
    dz = torch.where(torch.rand_like(dz) < 0.4, torch.zeros_like(dz), dz).to(torch.bfloat16)
    cf, dzf = c.float(), dz.float()
    M = B * H * H
    mean = cf.reshape(M, K).mean(0)
    rstd = torch.rsqrt(cf.reshape(M, K).var(0, unbiased=False) + 1e-5)
    gamma = torch.rand(K, device=dev) + 0.5
    xh = (cf - mean) * rstd
    # partial rows [G][dbeta (K) | dgamma (K)]: the pixel range cut into G pieces
    rows = []
    edges = torch.linspace(0, M, G + 1).long().tolist()
    d2, x2 = dzf.reshape(M, K), xh.reshape(M, K)
    for a, b in zip(edges[:-1], edges[1:]):
        rows.append(torch.cat([d2[a:b].sum(0), (d2[a:b] * x2[a:b]).sum(0)]))
    part = torch.stack(rows).contiguous()
    if not Kk.bnb_ok(x.shape, K, 3, 3, (1, 1), (1, 1), G):
        pytest.skip("no BN-folded pair for this shape's plans")
    dw = torch.full((K, 3, 3, C), 0.25, device=dev)
    dgam = torch.full((K,), 0.5, device=dev)
    dbet = torch.full((K,), -0.5, device=dev)
    dx = Kk.conv_bwd(dz, w, x, dw, 3, 3, (1, 1), (1, 1), accumulate=True,
                     bnb=(c, part, G, mean, rstd, gamma, dgam, dbet, acc))
    torch.cuda.synchronize()
    # fp32 reference of the same ops (dc rounded to bf16 as the kernel stages it)
    dbeta_r, dgamma_r = d2.sum(0), (d2 * x2).sum(0)
    dc = gamma * rstd * (dzf - dbeta_r / M - xh * dgamma_r / M)
    dc = dc.to(torch.bfloat16).float().permute(0, 3, 1, 2)
    xr, wr = x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2)
    dx_r = torch.nn.grad.conv2d_input(xr.shape, wr, dc, stride=1, padding=1).permute(0, 2, 3, 1)
    dw_r = torch.nn.grad.conv2d_weight(xr, wr.shape, dc, stride=1, padding=1).permute(0, 2, 3, 1)
    assert _rel(dx, dx_r) < 1e-2, _rel(dx, dx_r)
    assert _rel(dw - 0.25, dw_r) < 1e-2, _rel(dw - 0.25, dw_r)
    base_g, base_b = (0.5, -0.5) if acc else (0.0, 0.0)
    assert _rel(dgam - base_g, dgamma_r) < 1e-4
    assert _rel(dbet - base_b, dbeta_r) < 1e-4
