"""Bitwise-reproducible training steps (no atomics on any gradient path).

Every gradient producer of the CNN step writes each element once: conv weight gradients
sum their split-K partial tiles in split order (conv_igemm.hip), an unrolled 2x2-map conv
computes its weight gradient in the plain 3x3 form, BN dgamma/dbeta are summed from ordered
partial rows, and the fused cross-entropy bias gradient from ordered per-block rows
(loss.hip).  So two identical runs give identical bits, and the gradient buffer needs no
per-step memset: producers overwrite (nn/flat.py grad_out)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)


def _run(steps=4, model="resnet34", B=64):
    from kubeml_amd.engine.dp import make_train_step
    from kubeml_amd.models import resnet
    from kubeml_amd.nn import cross_entropy, flatten_module
    from kubeml_amd.ops import kernels as K
    from kubeml_amd.optim import SGD
    g = torch.Generator(device=dev).manual_seed(3)
    data = torch.randint(0, 256, (4096, 32, 32, 3), dtype=torch.uint8, device=dev, generator=g)
    labels = torch.randint(0, 10, (4096,), dtype=torch.int64, device=dev, generator=g)
    torch.manual_seed(1234)
    m = getattr(resnet, model)(num_classes=1000).to(dev)
    m.train()
    sp = flatten_module(m)
    opt = SGD(m.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    ctr = torch.tensor([1000.0, 0.0, 0.0], dtype=torch.float32, device=dev)
    x = torch.empty((B, 32, 32, 8), dtype=torch.bfloat16, device=dev)
    y = torch.empty((B,), dtype=torch.int64, device=dev)
    st = make_train_step(m, sp, opt, cross_entropy, x, y,
                         pre=lambda: K.augment(data, labels, ctr, B, out=x, labels_out=y, train=True),
                         advance=(ctr, B, 4096), extra_state=[ctr])
    st.capture()
    losses = [float(st()) for _ in range(steps)]
    torch.cuda.synchronize()
    return sp.state.clone(), sp.grad.clone(), losses


def test_two_identical_runs_are_bitwise_equal():
    s1, g1, l1 = _run()
    s2, g2, l2 = _run()
    assert l1 == l2, (l1, l2)
    assert torch.equal(g1, g2), float((g1 - g2).abs().max())
    assert torch.equal(s1, s2), float((s1 - s2).abs().max())    # master weights + BN statistics


def test_gradient_buffer_is_not_memset_every_step():
    """After the first step only add-only producers' regions are zeroed (ResNet-34 has none:
    every gradient is stored by its producer), and the result equals a full-zero run."""
    from kubeml_amd.nn.flat import FlatParamSpace
    s1, g1, _ = _run(steps=3)
    FlatParamSpace.full_zero = True
    try:
        s2, g2, _ = _run(steps=3)
    finally:
        FlatParamSpace.full_zero = False
    assert torch.equal(g1, g2) and torch.equal(s1, s2)
    from kubeml_amd.models.resnet import resnet34
    from kubeml_amd.nn import flatten_module
    m = resnet34(num_classes=1000).to(dev)
    sp = flatten_module(m)
    assert len(sp.params) > 100
