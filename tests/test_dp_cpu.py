"""Synchronous-DP (K=1) semantics and the bench launcher, on CPU.

* KubeModel with K=1 and an SGD optimizer runs rounds as gradient all-reduce
  (``self.step``); the reference averages WEIGHTS after each one-batch round and resets
  the optimizer state (python/kubeml/kubeml/network.py:276-310, 121-128).  The two must
  give the same model: checked with 2 thread-ranks against KUBEML_GRAD_SYNC=0 (the
  weight-averaging path), with momentum (reset every round) and weight decay.
* ``bench.py --gpus 2 --cpu-smoke`` launches 2 gloo ranks through torch.distributed.run
  and reports one JSON line with both ranks joined and in sync.
"""
import json
import os
import subprocess
import sys
import threading

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dataset(root):
    from kubeml_amd.store.shards import ShardStore
    rng = np.random.default_rng(0)
    st = ShardStore(root)
    if not st.exists("toy"):
        x = rng.integers(0, 255, (64 * 9 + 40, 28, 28)).astype(np.uint8)   # uneven shards, ragged last doc
        y = rng.integers(0, 10, len(x)).astype(np.int64)
        st.create("toy", x, y, x[:128], y[:128])
    return st


def _train_two_ranks(store_dir, grad_sync, epochs=2, momentum=0.9):
    from kubeml_amd.models.lenet import LeNet
    from kubeml_amd.parallel.comm import ThreadComm
    from kubeml_amd.sdk.context import TaskContext, reset_task, set_task
    from kubeml_amd.sdk.dataset import KubeDataset
    from kubeml_amd.sdk.model import KubeModel
    from kubeml_amd.store.shards import ShardStore

    class DS(KubeDataset):
        def __init__(self):
            super().__init__("toy")

        def __getitem__(self, i):
            return torch.from_numpy(self.data[i].astype(np.float32) / 255.0).unsqueeze(0), int(self.labels[i])

        def __len__(self):
            return len(self.data)

    class Net(KubeModel):
        def configure_optimizers(self):
            return torch.optim.SGD(self.parameters(), lr=0.05, momentum=momentum, weight_decay=1e-4)

        def train(self, batch, idx):
            x, y = batch
            return self.step(x, y, torch.nn.functional.cross_entropy)

    old = os.environ.get("KUBEML_GRAD_SYNC")
    os.environ["KUBEML_GRAD_SYNC"] = "1" if grad_sync else "0"
    comms = ThreadComm.create(2)
    store = ShardStore(store_dir)
    out, errs = [None, None], []
    nets = []
    for _ in range(2):          # the global RNG is shared by threads: initialise up front
        torch.manual_seed(0)
        nets.append(LeNet())

    def w(r):
        try:
            net = nets[r]
            km = None
            rounds = 0
            for e in range(1, epochs + 1):
                ctx = TaskContext(job_id="j", N=2, K=1, task="train", func_id=r, lr=0.05, batch_size=64, epoch=e,
                                  comm=comms[r], store=store, store_dir=store_dir)
                tok = set_task(ctx)
                try:
                    if km is None:
                        km = Net(net, DS())
                    km.start()
                    rounds += ctx.extra.get("grad_rounds", 0)
                finally:
                    reset_task(tok)
            sd = {k: v.detach().clone() for k, v in net.state_dict().items()}
            out[r] = (sd, rounds)
        except Exception as ex:  # pragma: no cover
            import traceback
            errs.append(traceback.format_exc())
    torch.set_num_threads(1)
    ts = [threading.Thread(target=w, args=(r,)) for r in range(2)]
    try:
        [t.start() for t in ts]
        [t.join() for t in ts]
    finally:
        if old is None:
            os.environ.pop("KUBEML_GRAD_SYNC", None)
        else:
            os.environ["KUBEML_GRAD_SYNC"] = old
    assert not errs, errs[0]
    return out


def test_k1_gradient_sync_equals_weight_average(tmp_path):
    _dataset(str(tmp_path))
    g = _train_two_ranks(str(tmp_path), grad_sync=True)
    a = _train_two_ranks(str(tmp_path), grad_sync=False)
    assert g[0][1] > 0 and a[0][1] == 0           # the grad-sync path really ran (and only there)
    for k in g[0][0]:
        # ranks agree with each other, and grad-sync agrees with the reference weight average
        t0, t1, ref = g[0][0][k].double(), g[1][0][k].double(), a[0][0][k].double()
        assert torch.allclose(t0, t1, atol=1e-6), k
        assert torch.allclose(t0, ref, rtol=1e-4, atol=2e-5), (k, float((t0 - ref).abs().max()))


def test_bench_cpu_smoke_launches_two_ranks():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--cpu-smoke", "--steps",
                        "3", "--warmup", "1"], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["ranks"] == 2 and d["ranks_joined"] == 2 and d["ranks_in_sync"] is True


def test_bench_rejects_more_gpus_than_visible():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 2 and "only 0 GPU" in r.stderr, (r.returncode, r.stderr[-2000:])


def _opt_overlap_run(opt_overlap, steps=3):
    from kubeml_amd.engine.dp import make_train_step
    from kubeml_amd.models.resnet import resnet18
    from kubeml_amd.nn import flatten_module
    from kubeml_amd.optim import SGD
    torch.manual_seed(0)
    m = resnet18(10)
    m.train()
    sp = flatten_module(m)
    opt = SGD(m.parameters(), lr=0.05, momentum=0.9, dampening=0.1, weight_decay=1e-4)
    x = torch.empty(4, 3, 32, 32)
    y = torch.empty(4, dtype=torch.int64)
    g = torch.Generator().manual_seed(5)

    def pre():
        x.copy_(torch.randn(4, 3, 32, 32, generator=g))
        y.copy_(torch.randint(0, 10, (4,), generator=g))
    step = make_train_step(m, sp, opt, torch.nn.functional.cross_entropy, x, y, pre=pre,
                           opt_overlap=opt_overlap)
    assert (step.segment_opt is not None) == opt_overlap
    losses = [float(step()) for _ in range(steps)]
    return sp.master.clone(), losses


def test_optimizer_overlapped_with_backward_matches_one_update():
    """opt_overlap: the update of each backward stage's parameter range runs as soon as the
    stage's gradients are final.  Same weights and losses as one optimizer step after the
    whole backward (momentum + dampening + weight decay, 3 steps)."""
    wa, la = _opt_overlap_run(True)
    wb, lb = _opt_overlap_run(False)
    assert la == pytest.approx(lb, rel=1e-6, abs=1e-6)
    torch.testing.assert_close(wa, wb, rtol=1e-5, atol=1e-6)


def test_comm_plan_parse_and_choice(tmp_path, monkeypatch):
    import json as _json
    from kubeml_amd.parallel.plan import CommPlan, choose_plan, parse_plan
    p = parse_plan("peer:overlap:bf16:32")
    assert (p.backend, p.schedule, p.wire, p.max_blocks) == ("peer", "overlap", "bf16", 32)
    assert p.tag() == "peer:overlap:bf16:32" and p.wire_dtype == torch.bfloat16
    assert parse_plan("rccl:end:fp32").tag() == "rccl:end:fp32"
    for bad in ("peer:end", "nccl:end:fp32", "peer:sometimes:fp32", "peer:end:fp16"):
        with pytest.raises(ValueError):
            parse_plan(bad)
    monkeypatch.delenv("KUBEML_COMM_PLAN", raising=False)
    table = {"choice": {"2": "peer:end:fp32:256", "8": "peer:overlap:bf16:64"}}
    assert choose_plan(8, 1 << 20, table=table).tag() == "peer:overlap:bf16:64"
    assert choose_plan(2, 1 << 20, table=table).tag() == "peer:end:fp32:256"
    assert choose_plan(6, 1 << 20, table=table).tag() == "peer:overlap:bf16:64"     # nearest N
    assert choose_plan(4, 1 << 20, table={}).source == "default"
    assert choose_plan(4, 1 << 20, gpu=False).backend == "rccl"
    monkeypatch.setenv("KUBEML_COMM_PLAN", "rccl:overlap:fp32")
    assert choose_plan(8, 1 << 20, table=table).tag() == "rccl:overlap:fp32"
    assert choose_plan(8, 1 << 20, override="peer:end:bf16:128", table=table).tag() == "peer:end:bf16:128"
    assert CommPlan().tag() == "peer:end:fp32:256"


def test_shipped_plan_table_is_exact_fp32():
    """The shipped table never picks a lossy wire by default (bf16 is opt-in)."""
    from kubeml_amd.parallel.plan import choose_plan
    for n in (2, 4, 8):
        assert choose_plan(n, 1 << 24).wire == "fp32"


def test_shipped_plan_rides_the_shard_step_when_it_predicts_faster(monkeypatch):
    """N > 1 defaults to the same-queue shard riders exactly where the probe's prediction beats
    the end-of-backward shard step (comm_plan.json shard_plans, tools/shard_plan_probe.py)."""
    import json as _json
    from kubeml_amd.parallel.plan import PLAN_FILE, choose_plan
    monkeypatch.delenv("KUBEML_COMM_PLAN", raising=False)
    table = _json.load(open(PLAN_FILE))
    for n in ("2", "4", "8"):
        pred = table["shard_plans"]["predicted_ms"][n]
        best = min(pred, key=pred.get)
        assert choose_plan(int(n), 1 << 24).tag() == best == table["choice"][n]
        assert pred["peer:shardride:fp32:1024"] < pred["peer:shard:fp32:1024"]


class _FakePeer:
    def __init__(self, poisoned=False, fits=True):
        self.poisoned, self.fits, self.released, self.closed = poisoned, fits, False, False
        self.region = object()

    def check(self):
        if self.poisoned:
            from kubeml_amd.parallel.peer import PeerCommError
            raise PeerCommError("barrier timeout")

    def supports(self, *a):
        return self.fits

    def _release(self):
        self.released = True

    def close(self):
        self.closed = True


def _bare_comm():
    from kubeml_amd.parallel.comm import TorchComm
    c = TorchComm.__new__(TorchComm)
    c.rank, c.world, c._subs, c.peer_data = 0, 2, {}, True
    c.peer = c.grad_peer = None
    return c


def test_poisoned_peer_is_dropped_and_the_next_job_recovers():
    """A barrier timeout poisons a transport for good; ``check()`` raises once, drops it
    (unmapped without a group barrier), and the following job's check passes — the next
    collective then builds a fresh transport instead of reusing the NaN one."""
    from kubeml_amd.parallel.peer import PeerCommError
    c = _bare_comm()
    sub = _bare_comm()
    c._subs[2] = sub
    bad, good = _FakePeer(poisoned=True), _FakePeer()
    c.peer, sub.grad_peer = good, bad
    with pytest.raises(PeerCommError):
        c.check()
    assert sub.grad_peer is None and bad.released and c.peer is good and not good.released
    c.check()                                     # next job: clean


def test_grad_peer_reused_only_if_it_fits():
    """A cached gradient transport is reused only when its slots fit this model's gradient
    at this wire; otherwise it is closed and a new one is built."""
    from kubeml_amd.parallel.plan import parse_plan
    from kubeml_amd.sdk.model import KubeModel
    km = KubeModel.__new__(KubeModel)
    km._flat = type("S", (), {"grad": torch.zeros(8)})()
    km._shards = {}
    c = _bare_comm()
    plan = parse_plan("peer:end:fp32:256")
    c.grad_peer = fit = _FakePeer(fits=True)
    assert km._reusable_peer(c, plan) is fit and c.grad_peer is fit
    c.grad_peer = small = _FakePeer(fits=False)
    assert km._reusable_peer(c, plan) is None and small.closed and c.grad_peer is None
    assert km._reusable_peer(c, parse_plan("rccl:end:fp32")) is None


def test_ride_plan_groups_and_rest_ranges(monkeypatch):
    """The SGD rider's plan (engine/dp.py ``ride``): ResNet groups from KUBEML_RIDE_PLAN, host convs
    disjoint per group, and the end-of-step ranges = the complement of the groups' flat ranges."""
    import pytest
    from kubeml_amd.engine.dp import ride_rest
    from kubeml_amd.models.resnet import resnet18, resnet50
    from kubeml_amd.nn import flatten_module
    m = resnet18(10)
    sp = flatten_module(m)
    monkeypatch.delenv("KUBEML_RIDE_PLAN", raising=False)
    (ps, hosts), (ps2, hosts2) = m.ride_plan()   # default "4f:321;123:s"
    assert {id(p) for p in ps} == {id(p) for p in list(m.layer4.parameters()) + list(m.fc.parameters())}
    assert len(hosts) == 5 + 5 + 4          # layer3 (with its downsample), layer2 (same), layer1
    assert {id(p) for p in ps2} == {id(p) for d in (1, 2, 3) for p in getattr(m, f"layer{d}").parameters()}
    assert [id(h) for h in hosts2] == [id(m.conv1)]   # the stem's weight-gradient launch
    lo, hi = sp.range_of(ps)
    lo2, hi2 = sp.range_of(ps2)
    assert lo == 0 and 0 < hi == lo2 < hi2 < sp.numel   # later layers sit first in the flat layout
    assert ride_rest([(lo, hi), (lo2, hi2)], sp.numel) == [(hi2, sp.numel)]   # the stem's own update
    monkeypatch.setenv("KUBEML_RIDE_PLAN", "4f:3;3:21")
    g = m.ride_plan()
    assert len(g) == 2 and not {id(h) for h in g[0][1]} & {id(h) for h in g[1][1]}
    r = [sp.range_of(p) for p, _ in g]
    assert ride_rest(r, sp.numel) == [(r[1][1], sp.numel)]
    assert ride_rest([(10, 20)], 30) == [(0, 10), (20, 30)]
    with pytest.raises(ValueError):
        ride_rest([(0, 20), (10, 30)], 40)
    monkeypatch.delenv("KUBEML_RIDE_PLAN", raising=False)
    assert resnet50(10).ride_plan() == []    # measured on BasicBlock nets only
