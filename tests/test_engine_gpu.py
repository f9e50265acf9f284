"""Training-engine semantics on the MI355X.

* ``KubeModel.step`` (graph per batch shape) applies exactly ONE optimizer update per
  call: capture's warm-up runs on snapshots, so batches of shapes (B, B, b_last, B)
  give the same master weights as the same number of eager fused-SGD steps — with
  momentum 0.9 / dampening 0.1 across a ``reset_state()`` (device first-step flag).
* K-AVG pack/finish kernels on the flat state buffer: divisor from the device count
  slot, bf16 shadow refresh, int64 counters floored back (reference integer division).
* ``bench.py`` end to end: the default path (timed steps + a measured epoch with
  validation) and the 1-rank RCCL rehearsal of the captured, overlapped all-reduce.
"""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _km(net, opt_fn):
    from kubeml_amd.nn import flatten_module
    from kubeml_amd.sdk.model import KubeModel

    class M(KubeModel):
        pass
    km = M(net, None, gpu=True)
    net.to(dev)
    km.device = dev
    km._flat = flatten_module(net)
    km.optimizer = opt_fn(net.parameters())
    return km


def _batches():
    g = torch.Generator(device=dev).manual_seed(7)
    shapes = [32, 32, 20, 32, 32]
    out = []
    for b in shapes:
        x = torch.randn(b, 32, 32, 8, device=dev, generator=g).to(torch.bfloat16)
        x[..., 3:] = 0
        y = torch.randint(0, 10, (b,), device=dev, generator=g)
        out.append((x, y))
    return out


def _pair_run(monkeypatch, lr, data, reset_at=3):
    from kubeml_amd.models.resnet import resnet18
    from kubeml_amd.optim import SGD

    def opt(ps):
        return SGD(ps, lr=lr, momentum=0.9, dampening=0.1, weight_decay=1e-4)
    torch.manual_seed(0)
    a = resnet18(10)
    b = resnet18(10)
    b.load_state_dict(a.state_dict())
    ka, kb = _km(a, opt), _km(b, opt)
    w0 = ka._flat.master.clone()

    def run(km, graph):
        if graph:
            monkeypatch.delenv("KUBEML_NO_GRAPH", raising=False)
        else:
            monkeypatch.setenv("KUBEML_NO_GRAPH", "1")
        losses = []
        for i, (x, y) in enumerate(data):
            if i == reset_at:
                km.optimizer.reset_state()     # K-AVG round boundary
            losses.append(float(km.step(x, y).detach()))
        torch.cuda.synchronize()
        return losses
    la = run(ka, graph=True)
    lb = run(kb, graph=False)
    return ka, kb, a, b, w0, la, lb


def test_graphed_step_first_update_matches_eager(monkeypatch):
    """One batch at a large LR: an extra warm-up update would move the weights by
    ~lr * |g| (~1e-2); the graph and eager paths agree to rounding."""
    ka, kb, a, b, w0, la, lb = _pair_run(monkeypatch, 0.05, _batches()[:1])
    upd = float((kb._flat.master - w0).abs().max())
    d = float((ka._flat.master - kb._flat.master).abs().max())
    assert upd > 1e-3 and d <= 1e-4 * upd, (d, upd)
    assert torch.equal(ka._flat.shadow, ka._flat.master.to(torch.bfloat16))


def test_graphed_step_applies_one_update_per_batch(monkeypatch):
    """Shapes (B, B, b_last, B, B) with momentum/dampening across reset_state(): the
    accumulated update equals the eager one: every gradient producer is deterministic, so
    graph and eager differ only by fp32 rounding of the update order."""
    data = _batches()
    ka, kb, a, b, w0, la, lb = _pair_run(monkeypatch, 1e-3, data)
    assert len(ka._graphs) == 2                # one graph per batch shape, re-used
    ua, ub = ka._flat.master - w0, kb._flat.master - w0
    rel = float((ua - ub).norm() / ub.norm())
    # every gradient producer is deterministic (no atomics): graph and eager replay the same
    # kernels, so the updates agree to fp32 rounding of the update order only
    assert rel <= 1e-5, (rel, la, lb)
    ratio = float(ua.norm() / ub.norm())
    assert 0.98 < ratio < 1.02, ratio          # 3 updates per batch would give ~3x
    for x, y in zip(la, lb):
        assert abs(x - y) <= 1e-2 * max(1.0, abs(y)), (la, lb)
    # BN running statistics and counters advanced once per batch, not per warm-up
    for (n, ba), (_, bb) in zip(a.named_buffers(), b.named_buffers()):
        if ba.dtype == torch.int64:
            assert int(ba) == int(bb) == len(data), n
        else:
            assert torch.allclose(ba, bb, rtol=1e-5, atol=1e-6), n


def test_kavg_pack_finish_kernels():
    from kubeml_amd.models.resnet import resnet18
    from kubeml_amd.nn import flatten_module
    from kubeml_amd.ops import kernels as K
    torch.manual_seed(0)
    net = resnet18(10).to(dev)
    sp = flatten_module(net)
    arena = sp.i64_arena_now()
    assert arena is not None and arena.numel() == sp.n_i64 > 0
    arena.copy_(torch.arange(sp.n_i64, device=dev) * 3 + 1)
    ref = sp.state[:sp.count_idx].clone()
    n = 3     # emulate the SUM all-reduce of 3 identical contributing ranks
    K.kavg_pack_(sp.state, arena, sp.i64_off, sp.n_i64, sp.count_idx, True)
    assert float(sp.state[sp.count_idx]) == 1.0
    sp.state.mul_(n)
    K.kavg_finish_(sp.state, sp.numel, sp.count_idx, sp.shadow, arena, sp.i64_off, sp.n_i64)
    got = sp.state[:sp.i64_off]
    assert torch.allclose(got, ref[:sp.i64_off], rtol=1e-6, atol=1e-7)
    assert torch.equal(sp.shadow, sp.master.to(torch.bfloat16))
    assert torch.equal(arena, torch.arange(sp.n_i64, device=dev) * 3 + 1)
    # mixed contributions: counters 1 and 4 over 2 ranks -> floor(5/2) = 2 (reference int division)
    arena.fill_(1)
    K.kavg_pack_(sp.state, arena, sp.i64_off, sp.n_i64, sp.count_idx, True)
    sp.state[sp.i64_off:sp.i64_off + sp.n_i64] += 4
    sp.state[sp.count_idx] += 1
    K.kavg_finish_(sp.state, sp.numel, sp.count_idx, sp.shadow, arena, sp.i64_off, sp.n_i64)
    assert torch.equal(arena, torch.full_like(arena, 2))
    # BN buffers are views into the state buffer
    bn = net.bn1
    lo, hi = sp.state.data_ptr(), sp.state.data_ptr() + 4 * sp.state.numel()
    assert lo <= bn.running_mean.data_ptr() < hi and lo <= bn.running_var.data_ptr() < hi


def _bench(*extra, timeout=600):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + list(extra), capture_output=True,
                       text=True, timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_measures_epoch_with_validation():
    d = _bench("--steps", "10", "--warmup", "2", "--batch", "128", "--e2e", "off")
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["epoch_measured"] is True
    assert d["val_images"] >= 10000 and d["epoch_time_s"] > d["epoch_train_s"] > 0
    assert d["loss_first_last"][1] == d["loss_first_last"][1]
    assert "e2e_epoch_time_s" not in d


def test_bench_reports_the_framework_epoch():
    """bench.py's default (N = 1) also runs the epoch through the whole stack: server, worker,
    storage upload, `kubeml train` with validation every epoch (experiments/e2e.py)."""
    d = _bench("--steps", "10", "--warmup", "2", "--e2e", "on", timeout=900)
    assert d.get("e2e_error") is None, d.get("e2e_error")
    assert d["e2e_epoch_time_s"] > 0 and len(d["e2e_epoch_wall_s"]) == 4 and d["e2e_warmup_epochs"] == 2
    assert d["e2e_total_s"] >= sum(d["e2e_epoch_wall_s"]) - 1e-3
    assert d["e2e_train_task_img_s"] > 0 and d["e2e_vs_bench_step_rate"] > 0


def test_bench_rccl_rehearsal_overlapped_graph_comm():
    d = _bench("--steps", "8", "--warmup", "2", "--batch", "128", "--force-comm", "--overlap", "on",
               "--no-epoch", "--comm-plan", "rccl:overlap:fp32")
    assert d["ranks_in_sync"] is True and d["config"]["overlap_segments"] is True
    assert d["config"]["graph_comm"] is True and d["rccl_world"] == 1


def test_bench_trace_has_compute_and_comm_tracks(tmp_path):
    """KUBEML_TRACE timeline: per-segment compute spans and per-segment all-reduce spans
    on their own tracks, device-timestamped, each all-reduce starting at its segment's end."""
    d = _bench("--steps", "3", "--warmup", "1", "--batch", "64", "--force-comm", "--overlap", "on", "--no-epoch",
               "--trace", str(tmp_path), "--comm-plan", "rccl:overlap:fp32")
    assert d["ranks_in_sync"] is True
    files = list(tmp_path.glob("*.json"))
    assert files
    evs = json.load(open(files[0]))["traceEvents"]
    comp = [e for e in evs if e.get("cat") == "gpu" and e["tid"] == 900001]
    comm = [e for e in evs if e.get("cat") == "gpu" and e["tid"] == 900002]
    assert len(comp) >= 3 * 4 and len(comm) >= 3 * 3
    seg_end = {}
    for e in comp:
        if "segment" in e["args"]:
            seg_end.setdefault(e["args"]["segment"], []).append(e["ts"] + e["dur"])
    for e in comm:
        ends = seg_end[e["args"]["segment"]]
        assert min(abs(e["ts"] - t) for t in ends) < 1.0   # starts where its segment ended
        assert e["dur"] >= 0


def _graphed_run(opt_overlap, steps=3, ride=False, arch="resnet18"):
    from kubeml_amd.engine.dp import make_train_step
    from kubeml_amd.models import resnet as R
    from kubeml_amd.nn import cross_entropy, flatten_module
    from kubeml_amd.optim import SGD
    torch.manual_seed(0)
    m = getattr(R, arch)(10).to(dev)
    m.train()
    sp = flatten_module(m)
    opt = SGD(m.parameters(), lr=1e-3, momentum=0.9, dampening=0.1, weight_decay=1e-4)
    g = torch.Generator(device=dev).manual_seed(11)
    xs = torch.randn(steps + 2, 32, 32, 32, 8, device=dev, generator=g).to(torch.bfloat16)
    xs[..., 3:] = 0
    ys = torch.randint(0, 10, (steps + 2, 32), device=dev, generator=g)
    x = torch.empty(32, 32, 32, 8, dtype=torch.bfloat16, device=dev)
    y = torch.empty(32, dtype=torch.int64, device=dev)
    i = torch.zeros((), dtype=torch.int64, device=dev)

    def pre():
        x.copy_(xs.index_select(0, i.view(1)).squeeze(0))
        y.copy_(ys.index_select(0, i.view(1)).squeeze(0))

    def post():
        i.add_(1)
    w0 = sp.master.clone()
    step = make_train_step(m, sp, opt, cross_entropy, x, y, pre=pre, post=post, opt_overlap=opt_overlap,
                           extra_state=[i], ride=ride)
    assert (step.segment_opt is not None) == opt_overlap
    step.capture()
    losses = [float(step()) for _ in range(steps)]
    torch.cuda.synchronize()
    return sp.master - w0, sp, losses


@pytest.mark.parametrize("arch,plan", [("resnet18", "4f:321"), ("resnet34", "4f:321"), ("resnet34", "4f:3;3:21"),
                                       ("resnet34", "4f:321;23:s"), ("resnet34", "4f:321;123:s")])
def test_ride_sgd_in_backward_launches_is_bit_exact(arch, plan, monkeypatch):
    """make_train_step(ride=True): the SGD (momentum, dampening, weight decay, first step after
    the reset) of layer4 + fc — and, with the two-group plan, of layer3 after its early gradient
    fold — runs in extra blocks of later layers' grouped conv-backward launches (k_conv_pair's
    rider role, the same element update as k_sgd: csrc/include/kml_sgd.h); the end-of-step
    launch covers the rest.  Bit-identical masters, momenta and shadows."""
    monkeypatch.setenv("KUBEML_RIDE_PLAN", plan)
    ua, spa, la = _graphed_run(False, ride=True, arch=arch)
    ub, spb, lb = _graphed_run(False, ride=False, arch=arch)
    assert float(ub.abs().max()) > 1e-5
    assert torch.equal(ua, ub)
    assert la == lb
    assert torch.equal(spa.shadow, spb.shadow)


def test_graphed_optimizer_overlap_matches_end_of_step_update():
    """make_train_step(opt_overlap=True): each backward stage's SGD range runs on a side
    stream inside the captured step.  Same updates as the single end-of-step SGD (to the
    split-K atomic-order noise of the weight gradients), shadow = bf16(master)."""
    ua, spa, la = _graphed_run(True)
    ub, spb, lb = _graphed_run(False)
    assert float(ub.abs().max()) > 1e-5
    rel = float((ua - ub).norm() / ub.norm())
    assert rel <= 1e-5, rel
    for p, q in zip(la, lb):
        assert abs(p - q) <= 1e-3 * max(1.0, abs(q)), (la, lb)
    assert torch.equal(spa.shadow, spa.master.to(torch.bfloat16))


def _vgg_adam_run(overlap, steps=3):
    from kubeml_amd.engine.dp import make_train_step
    from kubeml_amd.models.vgg import vgg11_bn
    from kubeml_amd.nn import cross_entropy, flatten_module
    from kubeml_amd.optim import AdamW
    torch.manual_seed(0)
    net = vgg11_bn(100, dropout=0.0).to(dev)    # no dropout: the two capture paths warm up a
    net.train()                                   # different number of times (device RNG counter)
    sp = flatten_module(net)
    opt = AdamW(net.parameters(), lr=1e-3, weight_decay=0.01)
    w0 = sp.master.clone()
    g = torch.Generator(device=dev).manual_seed(3)
    xs = [torch.randn(32, 32, 32, 8, device=dev, generator=g).to(torch.bfloat16) for _ in range(steps)]
    ys = [torch.randint(0, 100, (32,), device=dev, generator=g) for _ in range(steps)]
    xb, yb = torch.empty_like(xs[0]), torch.empty_like(ys[0])
    step = make_train_step(net, sp, opt, cross_entropy, xb, yb, opt_overlap=overlap)
    step.capture()
    losses = []
    for x, y in zip(xs, ys):
        xb.copy_(x)
        yb.copy_(y)
        losses.append(float(step()))
    torch.cuda.synchronize()
    return sp.master - w0, sp, opt, losses, step


def test_graphed_adam_overlap_advances_the_step_once():
    """make_train_step(opt_overlap=True) with AdamW on VGG's [features, classifier] stages: the
    classifier's update runs on a side stream while the convolutions run backward.  The bias-
    correction step advances once per step (begin_ranges), so three overlapped steps equal three
    end-of-step updates (to split-K atomic-order noise) and the device counter reads 3."""
    ua, spa, oa, la, sa = _vgg_adam_run(True)
    ub, spb, ob, lb, sb = _vgg_adam_run(False)
    assert sa.segment_opt is not None and sb.segment_opt is None
    assert float(oa.step_tensor(dev)) == float(ob.step_tensor(dev)) == 3.0
    assert float(ub.abs().max()) > 1e-5
    rel = float((ua - ub).norm() / ub.norm())
    assert rel <= 1e-4, rel
    for p, q in zip(la, lb):
        assert abs(p - q) <= 1e-3 * max(1.0, abs(q)), (la, lb)
    assert torch.equal(spa.shadow, spa.master.to(torch.bfloat16))


def test_bench_peer_plans_rehearsal():
    """The peer transport inside the captured step (1-rank group: copy-in, reduce-scatter and
    all-gather kernels run; the link does not): end of step and overlapped with a block cap,
    fp32 and bf16 wire; the device-stamped all-reduce time is reported."""
    for spec in ("peer:end:fp32:256", "peer:overlap:bf16:32"):
        d = _bench("--steps", "30", "--warmup", "2", "--batch", "128", "--force-comm", "--no-epoch",
                   "--comm-plan", spec, "--comm-timing", "5")
        assert d["ranks_in_sync"] is True and d["config"]["comm_plan"] == spec, d
        assert d["config"]["overlap_segments"] is (":overlap:" in spec)
        assert d["allreduce_ms"] > 0, d
        assert d["loss_first_last"][1] == d["loss_first_last"][1]


def _plan_run(spec, steps=3):
    """_graphed_run's workload through make_train_step with a comm plan on a 1-rank group."""
    import torch.distributed as dist
    from kubeml_amd.engine.dp import make_train_step
    from kubeml_amd.models.resnet import resnet18
    from kubeml_amd.nn import cross_entropy, flatten_module
    from kubeml_amd.optim import SGD
    from kubeml_amd.parallel.plan import parse_plan
    from kubeml_amd.runtime.pool import free_port
    own = not dist.is_initialized()
    if own:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1)
    try:
        torch.manual_seed(0)
        m = resnet18(10).to(dev)
        m.train()
        sp = flatten_module(m)
        opt = SGD(m.parameters(), lr=1e-3, weight_decay=1e-4)
        g = torch.Generator(device=dev).manual_seed(11)
        xs = torch.randn(steps + 2, 32, 32, 32, 8, device=dev, generator=g).to(torch.bfloat16)
        xs[..., 3:] = 0
        ys = torch.randint(0, 10, (steps + 2, 32), device=dev, generator=g)
        x = torch.empty(32, 32, 32, 8, dtype=torch.bfloat16, device=dev)
        y = torch.empty(32, dtype=torch.int64, device=dev)
        i = torch.zeros((), dtype=torch.int64, device=dev)

        def pre():
            x.copy_(xs.index_select(0, i.view(1)).squeeze(0))
            y.copy_(ys.index_select(0, i.view(1)).squeeze(0))

        def post():
            i.add_(1)
        w0 = sp.master.clone()
        plan = parse_plan(spec) if spec else None
        step = make_train_step(m, sp, opt, cross_entropy, x, y, pre=pre, post=post, extra_state=[i],
                               plan=plan, force_comm=plan is not None, world=1)
        step.capture()
        losses = [float(step()) for _ in range(steps)]
        torch.cuda.synchronize()
        if step.peer is not None:
            step.peer.check()
            step.peer.close()
        return sp.master - w0, losses
    finally:
        if own:
            dist.destroy_process_group()


def test_peer_plans_on_one_rank_match_the_local_step():
    """World 1: the fp32 peer all-reduce is the identity (bitwise the same updates as no comm:
    every gradient producer is deterministic); the bf16 wire rounds the gradient to bf16."""
    ub, lb = _plan_run(None)
    for spec in ("peer:end:fp32:256", "peer:overlap:fp32:16"):
        ua, la = _plan_run(spec)
        assert torch.equal(ua, ub) and la == lb, (spec, float((ua - ub).abs().max()), la, lb)
    # one step (later steps amplify any perturbation chaotically through batch-32 BN over
    # 1x1 maps): the update differs only by the bf16 rounding of the gradient (2^-9 relative)
    ua, _ = _plan_run("peer:end:bf16:256", steps=1)
    ub1, _ = _plan_run(None, steps=1)
    rel = float((ua - ub1).norm() / ub1.norm())
    assert 0 < rel < 1e-2, rel
