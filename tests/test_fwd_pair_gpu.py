"""Forward pairs (conv_igemm.hip k_conv_fwd_pair, ops.kernels.conv_fwd_pair): the strided 3x3
conv and the 1x1 projection of ResNet-34/CIFAR's downsampling blocks (layer2/3/4 at batch 256)
launched as one kernel give bit-for-bit the outputs and BN partial-statistics rows of the two
separate launches, and those match fp32 torch."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)

# (H, Cin, Cout): the input map of each downsampling block at 32x32 images with the ImageNet stem
BLOCKS = [(8, 64, 128), (4, 128, 256), (2, 256, 512)]


def _convs(H, C, K, group):
    from kubeml_amd.ops import kernels as K_
    torch.manual_seed(H)
    x = torch.randn(256, H, H, C, device=dev).to(torch.bfloat16)
    w3 = (torch.randn(K, 3, 3, C, device=dev) * (9 * C) ** -0.5).to(torch.bfloat16)
    w1 = (torch.randn(K, 1, 1, C, device=dev) * C ** -0.5).to(torch.bfloat16)
    specs = [(w3, 3, (2, 2), (1, 1), group), (w1, 1, (2, 2), (0, 0), False)]
    outs = []
    for w, k, st, pd, grp in specs:
        G = K_.conv_fwd_stats_rows(x.shape, K, k, k, st, pd, group=grp)
        outs.append((x, w, k, st, pd, grp, torch.full((G * 2 * K,), float("nan"), device=dev)))
    return outs


def _run(convs):
    from kubeml_amd.ops import kernels as K_
    return [(K_.conv_fwd(x, w, k, k, st, pd, stats=rows, stats_part=True, stats_group=grp), rows)
            for x, w, k, st, pd, grp, rows in convs]


@pytest.mark.parametrize("H,C,K", BLOCKS)
@pytest.mark.parametrize("group", [False, True])
def test_forward_pair_matches_separate_launches(H, C, K, group):
    from kubeml_amd.ops import kernels as K_
    sep = _run(_convs(H, C, K, group))
    convs = _convs(H, C, K, group)
    n0 = K_.FWD_PAIRS_LAUNCHED[0]
    with K_.conv_fwd_pair():
        par = _run(convs)
    torch.cuda.synchronize()
    assert K_.FWD_PAIRS_LAUNCHED[0] == n0 + 1, "the two convs did not launch as a pair"
    for (ys, rs), (yp, rp) in zip(sep, par):
        assert torch.equal(ys, yp)
        assert torch.equal(torch.nan_to_num(rs, 7.0), torch.nan_to_num(rp, 7.0))
    x = convs[0][0].float().permute(0, 3, 1, 2)
    for (x_, w, k, st, pd, _, _), (y, _) in zip(convs, par):
        ref = F.conv2d(x, w.float().permute(0, 3, 1, 2), stride=st, padding=pd).permute(0, 2, 3, 1)
        assert float((y.float() - ref).abs().max() / ref.abs().max()) < 1e-2


def test_unpaired_plans_launch_separately():
    """Two convs whose plans are not an instantiated pair launch on their own, same results."""
    from kubeml_amd.ops import kernels as K_
    torch.manual_seed(0)
    x = torch.randn(8, 8, 8, 64, device=dev).to(torch.bfloat16)
    w = (torch.randn(64, 3, 3, 64, device=dev) * 0.05).to(torch.bfloat16)
    ref = K_.conv_fwd(x, w, 3, 3, (1, 1), (1, 1))
    n0 = K_.FWD_PAIRS_LAUNCHED[0]
    with K_.conv_fwd_pair():
        a = K_.conv_fwd(x, w, 3, 3, (1, 1), (1, 1))
        b = K_.conv_fwd(x, w, 3, 3, (1, 1), (1, 1))
    torch.cuda.synchronize()
    assert K_.FWD_PAIRS_LAUNCHED[0] == n0
    assert torch.equal(a, ref) and torch.equal(b, ref)


def test_resnet34_paired_downsampling_blocks_match_unpaired():
    """A ResNet-34 training forward + backward at batch 256 (the shapes the pairs are instantiated
    for) with the downsampling blocks' conv pairs (layers 2-4), BN-apply pairs (layers 3-4) and
    BN-backward apply pairs (layers 2-4) against
    the same step launched one kernel each: logits, loss, every gradient and the paired BNs'
    running statistics bit-identical."""
    from kubeml_amd.models.resnet import resnet34
    from kubeml_amd.nn import cross_entropy, flatten_module
    from kubeml_amd.nn import fused
    from kubeml_amd.ops import kernels as K_
    torch.manual_seed(0)
    x = torch.randn(256, 32, 32, 8, device=dev).to(torch.bfloat16)
    y = torch.randint(0, 1000, (256,), device=dev)
    old = fused._FWD_PAIR, fused._BWD_PAIR
    res, counts = [], []
    try:
        for on in (False, True):
            fused._FWD_PAIR = fused._BWD_PAIR = on
            c0 = (K_.FWD_PAIRS_LAUNCHED[0], K_.BN_PAIRS_LAUNCHED[0], K_.BNB_PAIRS[0])
            torch.manual_seed(3)
            m = resnet34(1000).to(dev)
            sp = flatten_module(m)
            m.train()
            sp.zero_grad()
            out = m(x)
            loss = cross_entropy(out, y)
            loss.backward()
            torch.cuda.synchronize()
            counts.append((K_.FWD_PAIRS_LAUNCHED[0] - c0[0], K_.BN_PAIRS_LAUNCHED[0] - c0[1], K_.BNB_PAIRS[0] - c0[2]))
            bns = [m.layer2[0].downsample[1], m.layer3[0].bn1, m.layer3[0].downsample[1], m.layer4[0].bn1,
                   m.layer4[0].downsample[1]]
            res.append((out.float(), float(loss), sp.grad.clone(),
                        [torch.cat([b.running_mean, b.running_var]) for b in bns]))
    finally:
        fused._FWD_PAIR, fused._BWD_PAIR = old
    # backward: the projection BN and the first BN of each downsampling block share one apply launch
    assert counts == [(0, 0, 0), (3, 2, 3)], counts
    (o0, l0, g0, r0), (o1, l1, g1, r1) = res
    assert torch.equal(o1, o0) and l1 == l0
    assert torch.equal(g1, g0)
    assert all(torch.equal(a, b) for a, b in zip(r0, r1))
