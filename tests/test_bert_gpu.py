"""BERT MLM on the MI355X kernels vs the same modules' fp64 CPU path, plus a
graph-captured Adam training loop (loss must fall on a memorisable batch)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _data(B, L, P, V, seed=0):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, V, (B, L), generator=g)
    tt = torch.randint(0, 2, (B, L), generator=g)
    pos = torch.stack([torch.randperm(L, generator=g)[:P].sort().values for _ in range(B)])
    lab = torch.randint(0, V, (B, P), generator=g)
    mask = torch.ones(B, L, dtype=torch.int64)
    mask[0, L - 5:] = 0
    return ids, tt, pos, lab, mask


def test_bert_tiny_matches_fp64():
    from kubeml_amd.models.bert import bert_tiny_mlm
    from kubeml_amd.nn import flatten_module
    torch.manual_seed(0)
    ref = bert_tiny_mlm(dropout=0.0).double()
    gpu = bert_tiny_mlm(dropout=0.0)
    gpu.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    gpu = gpu.to(dev)
    flatten_module(gpu)
    ids, tt, pos, lab, mask = _data(2, 128, 20, 1000)
    ref.train()
    gpu.train()
    lr = ref(ids, tt, mask, pos, lab)
    lr.backward()
    lg = gpu(ids.to(dev), tt.to(dev), mask.to(dev), pos.to(dev), lab.to(dev))
    lg.backward()
    assert abs(lg.item() - lr.item()) < 0.02 * abs(lr.item())
    pr = dict(ref.named_parameters())
    for name, p in gpu.named_parameters():
        e = _rel(p.grad.cpu(), pr[name].grad)
        assert e < 0.08, (name, e)
    # logits of the eval path
    gpu.eval()
    ref.eval()
    with torch.no_grad():
        zo = gpu(ids.to(dev), tt.to(dev), mask.to(dev), pos.to(dev))
        zr = ref(ids, tt, mask, pos)
    assert _rel(zo.float().cpu(), zr) < 0.02


def test_bert_tiny_graphed_adam_learns():
    from kubeml_amd.engine.step import GraphedTrainStep
    from kubeml_amd.models.bert import bert_tiny_mlm
    from kubeml_amd.nn import flatten_module
    from kubeml_amd.optim import AdamW
    torch.manual_seed(0)
    m = bert_tiny_mlm().to(dev)
    sp = flatten_module(m)
    m.train()
    opt = AdamW(m.parameters(), lr=2e-3, weight_decay=0.01)
    ids, tt, pos, lab, mask = (t.to(dev) for t in _data(4, 128, 20, 1000, seed=1))

    def fb():
        sp.zero_grad()
        loss = m(ids, tt, mask, pos, lab)
        loss.backward()
        return loss
    step = GraphedTrainStep(fb, opt.step, warmup=2)
    step.capture()
    first = None
    for i in range(60):
        l = step()
        if i == 0:
            first = float(l)
    last = float(l)
    assert first > 4.0 and last < 0.5 * first, (first, last)  # 3 steps already taken by warmup+capture


@pytest.mark.parametrize("dropout", [0.0, 0.1])
def test_bert_fused_residual_and_bias_gradients_match_unfused(dropout):
    """Residual-gradient sums in the dgrad epilogue and the out-projection / FFN2 bias
    gradients summed inside the LayerNorm backward (_RES_FUSE, default on) give the
    same loss and gradients as autograd adds + column-sum kernels (same dropout masks)."""
    from kubeml_amd.models.bert import bert_tiny_mlm
    from kubeml_amd.nn import flatten_module
    from kubeml_amd.nn import transformer as TR
    ids, tt, pos, lab, mask = _data(2, 128, 20, 1000, seed=3)
    out = []
    old = TR._RES_FUSE
    try:
        for fuse in (False, True):
            TR._RES_FUSE = fuse
            torch.manual_seed(0)
            TR.Dropout._salt = 0            # same per-layer salts (dropout masks) in both models
            m = bert_tiny_mlm(dropout=dropout).to(dev)
            sp = flatten_module(m)
            m.train()
            sp.zero_grad()
            loss = m(ids.to(dev), tt.to(dev), mask.to(dev), pos.to(dev), lab.to(dev))
            loss.backward()
            torch.cuda.synchronize()
            out.append((float(loss), sp.grad.clone(), {n: p.grad.clone() for n, p in m.named_parameters()}))
    finally:
        TR._RES_FUSE = old
    (l0, g0, p0), (l1, g1, p1) = out
    assert l1 == l0
    assert _rel(g1, g0) < 1e-3, _rel(g1, g0)
    for n in p0:
        if n.endswith("bias"):
            assert _rel(p1[n], p0[n]) < 1e-2, (n, _rel(p1[n], p0[n]))


def test_bert_ffn_gelu_backward_in_dgrad_epilogue_matches_unfused(monkeypatch):
    """FFN2's dgrad applying FFN1's GELU backward and summing FFN1's bias gradient in its
    epilogue (modules._GELU_FUSE, the 256x256 phase tile) == the separate GELU backward pass:
    same loss, the same weight gradients, bias gradients to fp32 summation order."""
    from kubeml_amd.models.bert import bert_tiny_mlm
    from kubeml_amd.nn import flatten_module
    from kubeml_amd.nn import modules as MO
    from kubeml_amd.nn import transformer as TR
    from kubeml_amd.ops import gemm as G
    orig = G.plan

    def plan(layout, M, N, K):   # force the phase tile on the tiny model's FFN2 dgrad
        if layout == 1 and N % 256 == 0 and N > K:
            return (256, 256, 8), 1
        return orig(layout, M, N, K)
    monkeypatch.setattr(G, "plan", plan)
    calls = []
    real = G.linear_dgrad_gelu

    def spy(*a, **k):
        r = real(*a, **k)
        calls.append(r is not None)
        return r
    monkeypatch.setattr(G, "linear_dgrad_gelu", spy)
    # large enough for the gemm.hip route of every Linear (>= 2048 tokens, >= 256 features)
    ids, tt, pos, lab, mask = _data(16, 128, 20, 1000, seed=4)
    out = []
    old = MO._GELU_FUSE
    try:
        for fuse in (False, True):
            MO._GELU_FUSE = fuse
            torch.manual_seed(0)
            TR.Dropout._salt = 0
            m = bert_tiny_mlm(dropout=0.1, hidden=256, inter=1024, heads=4).to(dev)
            sp = flatten_module(m)
            m.train()
            sp.zero_grad()
            loss = m(ids.to(dev), tt.to(dev), mask.to(dev), pos.to(dev), lab.to(dev))
            loss.backward()
            torch.cuda.synchronize()
            out.append((float(loss), {n: p.grad.clone() for n, p in m.named_parameters()}))
    finally:
        MO._GELU_FUSE = old
    assert calls and all(calls), calls
    (l0, p0), (l1, p1) = out
    assert l1 == l0
    for n in p0:
        if n.endswith("bias") or "embeddings" in n:   # fp32 order / atomic scatter-adds
            assert _rel(p1[n], p0[n]) < 1e-3, (n, _rel(p1[n], p0[n]))
        else:
            assert torch.equal(p1[n], p0[n]), n
