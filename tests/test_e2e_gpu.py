"""End-to-end on an MI355X: the server with a GPU worker trains the ResNet-34 CIFAR
function (HIP kernels, on-device augmentation, graphed step), validates, checkpoints
and serves inference from the checkpoint."""
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_resnet34_function_on_gpu_worker(tmp_path):
    from kubeml_amd.api.types import InferRequest, TrainOptions, TrainRequest
    from kubeml_amd.client import KubemlClient
    from kubeml_amd.config import Config
    from kubeml_amd.control.server import KubeMLServer
    cfg = Config()
    cfg.store_dir = str(tmp_path / "store")
    srv = KubeMLServer(cfg, n_workers=1, use_gpu=True, task_timeout=600).start(
        ports={k: 0 for k in ("controller", "scheduler", "ps", "storage", "metrics")})
    try:
        c = KubemlClient(srv.url())
        rng = np.random.default_rng(0)
        arrs = {"xtr": rng.integers(0, 256, (1280, 32, 32, 3), dtype=np.uint8),
                "ytr": rng.integers(0, 10, 1280).astype(np.int64),
                "xte": rng.integers(0, 256, (256, 32, 32, 3), dtype=np.uint8),
                "yte": rng.integers(0, 10, 256).astype(np.int64)}
        paths = {}
        for k, v in arrs.items():
            paths[k] = str(tmp_path / f"{k}.npy")
            np.save(paths[k], v)
        c.datasets.create("cifar10", paths["xtr"], paths["ytr"], paths["xte"], paths["yte"])
        c.functions.create("resnet34", os.path.join(ROOT, "examples", "function_resnet34.py"))
        jid = c.networks.train(TrainRequest(batch_size=128, epochs=2, dataset="cifar10", lr=0.05,
                                            function_name="resnet34",
                                            options=TrainOptions(default_parallelism=1, static_parallelism=True,
                                                                 validate_every=1, k=-1)))
        t0 = time.time()
        while c.tasks.status(jid)["state"] == "running":
            assert time.time() - t0 < 600
            time.sleep(0.5)
        st = c.tasks.status(jid)
        assert st["state"] == "finished", (st, c.logs(jid).decode()[-3000:])
        h = c.histories.get(jid).data
        assert len(h.train_loss) == 2 and all(np.isfinite(h.train_loss))
        assert len(h.accuracy) == 2 and all(0 <= a <= 100 for a in h.accuracy)
        out = c.networks.infer(InferRequest(model_id=jid, data=arrs["xte"][:3].tolist()))
        preds = out["predictions"]
        assert len(preds) == 3 and all(0 <= p < 1000 for p in preds)
    finally:
        srv.stop()


def _train_function(tmp_path, fn_name, fn_file, ds_name, arrs, batch, epochs, k, lr, workers=1, parallelism=1):
    """Upload ``arrs`` (xtr, ytr, xte, yte) as ``ds_name``, register ``fn_file`` and run
    ``kubeml train`` through the controller; returns (client, job id, history)."""
    from kubeml_amd.api.types import TrainOptions, TrainRequest
    from kubeml_amd.client import KubemlClient
    from kubeml_amd.config import Config
    from kubeml_amd.control.server import KubeMLServer
    cfg = Config()
    cfg.store_dir = str(tmp_path / "store")
    srv = KubeMLServer(cfg, n_workers=workers, use_gpu=True, task_timeout=600).start(
        ports={k_: 0 for k_ in ("controller", "scheduler", "ps", "storage", "metrics")})
    try:
        c = KubemlClient(srv.url())
        paths = {}
        for key, v in arrs.items():
            paths[key] = str(tmp_path / f"{key}.npy")
            np.save(paths[key], v)
        c.datasets.create(ds_name, paths["xtr"], paths["ytr"], paths["xte"], paths["yte"])
        c.functions.create(fn_name, os.path.join(ROOT, "examples", fn_file))
        jid = c.networks.train(TrainRequest(batch_size=batch, epochs=epochs, dataset=ds_name, lr=lr,
                                            function_name=fn_name,
                                            options=TrainOptions(default_parallelism=parallelism,
                                                                 static_parallelism=True, validate_every=1, k=k)))
        t0 = time.time()
        while c.tasks.status(jid)["state"] == "running":
            assert time.time() - t0 < 600
            time.sleep(0.5)
        st = c.tasks.status(jid)
        assert st["state"] == "finished", (st, c.logs(jid).decode()[-3000:])
        return c, jid, c.histories.get(jid).data
    finally:
        srv.stop()


def test_resnet50_kavg_function_on_gpu_worker(tmp_path):
    """Config 3 through KubeML: ImageNet-shaped uint8 images, K = 2 local steps per average."""
    rng = np.random.default_rng(1)
    arrs = {"xtr": rng.integers(0, 256, (128, 224, 224, 3), dtype=np.uint8),
            "ytr": rng.integers(0, 1000, 128).astype(np.int64),
            "xte": rng.integers(0, 256, (64, 224, 224, 3), dtype=np.uint8),
            "yte": rng.integers(0, 1000, 64).astype(np.int64)}
    _, _, h = _train_function(tmp_path, "resnet50", "function_resnet50.py", "imagenet_synth", arrs, batch=32,
                              epochs=2, k=2, lr=0.05)
    assert len(h.train_loss) == 2 and all(np.isfinite(h.train_loss))
    assert len(h.accuracy) == 2 and all(0 <= a <= 100 for a in h.accuracy)


def test_bert_mlm_function_on_gpu_worker(tmp_path):
    """Config 5 through KubeML: int64 token ids uploaded via the storage API, masked on device."""
    rng = np.random.default_rng(2)
    L = 128
    arrs = {"xtr": rng.integers(1000, 30000, (128, L)).astype(np.int64),
            "ytr": np.zeros(128, dtype=np.int64),
            "xte": rng.integers(1000, 30000, (64, L)).astype(np.int64),
            "yte": np.zeros(64, dtype=np.int64)}
    _, _, h = _train_function(tmp_path, "bert", "function_bert.py", "wiki_tokens", arrs, batch=16,
                              epochs=2, k=-1, lr=1e-4)
    assert len(h.train_loss) == 2 and all(np.isfinite(h.train_loss))
    assert h.train_loss[0] > 5.0                   # ~ln(30522) at random init
    assert len(h.accuracy) == 2 and all(0 <= a <= 100 for a in h.accuracy)


def _packed_server(tmp_path, workers, policy=None):
    """A server whose ``workers`` worker slots all run on the box's one GPU (reference packing,
    ``func_id % device_count``): the pool bootstraps over gloo and moves data through the
    peer-memory transport, since RCCL refuses two ranks on one device."""
    from kubeml_amd.config import Config
    from kubeml_amd.control.server import KubeMLServer
    cfg = Config()
    cfg.store_dir = str(tmp_path / "store")
    cfg.num_gpus = 1
    return KubeMLServer(cfg, n_workers=workers, use_gpu=True, task_timeout=600, policy=policy).start(
        ports={k_: 0 for k_ in ("controller", "scheduler", "ps", "storage", "metrics")})


def _cifar_like(n=1280, nte=256, seed=3):
    rng = np.random.default_rng(seed)
    return {"xtr": rng.integers(0, 256, (n, 32, 32, 3), dtype=np.uint8),
            "ytr": rng.integers(0, 10, n).astype(np.int64),
            "xte": rng.integers(0, 256, (nte, 32, 32, 3), dtype=np.uint8),
            "yte": rng.integers(0, 10, nte).astype(np.int64)}


def _run_job(c, tmp_path, k, parallelism, static=True, epochs=2, batch=128):
    import json
    from kubeml_amd.api.types import TrainOptions, TrainRequest
    jid = c.networks.train(TrainRequest(batch_size=batch, epochs=epochs, dataset="cifar10", lr=0.05,
                                        function_name="resnet34",
                                        options=TrainOptions(default_parallelism=parallelism,
                                                             static_parallelism=static, validate_every=1, k=k)))
    t0 = time.time()
    while c.tasks.status(jid)["state"] == "running":
        assert time.time() - t0 < 600
        time.sleep(0.5)
    st = c.tasks.status(jid)
    assert st["state"] == "finished", (st, c.logs(jid).decode()[-3000:])
    logs = [json.loads(l) for l in c.logs(jid).decode().splitlines() if l.startswith("{")]
    return jid, c.histories.get(jid).data, [l for l in logs if l.get("msg") == "epoch finished"]


def _same_model(ep):
    ck = list(ep["checksums"].values())
    ends = [v[1] for v in ck]
    return max(ends) - min(ends) <= 1e-6 * max(1.0, abs(ends[0]))


def test_two_workers_share_one_gpu_grad_sync_and_kavg(tmp_path):
    """``kubeml train --parallelism 2`` with both workers on the one GPU: K = 1 runs as the
    in-graph gradient sync (the comm plan's transport over peer memory), K = 4 as K-AVG
    rounds over the peer all-reduce; both keep the two workers on one model."""
    from kubeml_amd.client import KubemlClient
    srv = _packed_server(tmp_path, 2)
    try:
        assert srv.ps.n_gpus == 1 and srv.ps.inventory.n == 2
        c = KubemlClient(srv.url())
        arrs = _cifar_like()
        paths = {}
        for key, v in arrs.items():
            paths[key] = str(tmp_path / f"{key}.npy")
            np.save(paths[key], v)
        c.datasets.create("cifar10", paths["xtr"], paths["ytr"], paths["xte"], paths["yte"])
        c.functions.create("resnet34", os.path.join(ROOT, "examples", "function_resnet34.py"))
        for k, mode in ((1, "grad-allreduce"), (4, "kavg")):
            _, h, eps = _run_job(c, tmp_path, k, 2)
            assert h.parallelism == [2.0, 2.0] and all(np.isfinite(h.train_loss)), h
            assert all(m == mode for m in h.sync_mode), h.sync_mode
            assert all(len(e["checksums"]) == 2 and _same_model(e) for e in eps), eps
    finally:
        srv.stop()


def test_elastic_one_two_one_on_one_gpu(tmp_path):
    """Scripted elastic resize P = 1 -> 2 -> 1 with two workers on one GPU: the worker joining
    at P = 2 starts from rank 0's model (epoch-start broadcast over the peer transport) and both
    end the epoch on one model."""
    from kubeml_amd.client import KubemlClient
    srv = _packed_server(tmp_path, 2, policy="scripted:1,2,1")
    try:
        c = KubemlClient(srv.url())
        arrs = _cifar_like(seed=4)
        paths = {}
        for key, v in arrs.items():
            paths[key] = str(tmp_path / f"{key}.npy")
            np.save(paths[key], v)
        c.datasets.create("cifar10", paths["xtr"], paths["ytr"], paths["xte"], paths["yte"])
        c.functions.create("resnet34", os.path.join(ROOT, "examples", "function_resnet34.py"))
        _, h, eps = _run_job(c, tmp_path, 1, 1, static=False, epochs=3)
        assert h.parallelism == [1.0, 2.0, 1.0], h.parallelism
        assert [len(e["checksums"]) for e in eps] == [1, 2, 1]
        prev_end = None
        for e in eps:
            ck = list(e["checksums"].values())
            starts = [v[0] for v in ck]
            assert max(starts) - min(starts) <= 1e-9 * max(1.0, abs(starts[0])), e["checksums"]
            if prev_end is not None:
                assert abs(starts[0] - prev_end) <= 1e-6 * max(1.0, abs(prev_end)), (starts, prev_end)
            assert _same_model(e), e["checksums"]
            prev_end = ck[0][1]
    finally:
        srv.stop()


def test_bert_grad_sync_persistent_adamw_two_packed_workers(tmp_path):
    """Config 5 as a framework workload: ``kubeml train -f bert --K 1 --grad-sync --parallelism 2``
    with both workers packed on the one GPU.  K = 1 rounds run as the in-graph gradient exchange
    (the comm plan's transport over peer memory) with the AdamW moments kept across rounds
    (TrainOptions.sync = "grad"); masking, forward, backward and AdamW of a batch are one graph
    replay.  Both workers must end every epoch on one model, and the loss must fall."""
    import json
    from kubeml_amd.api.types import TrainOptions, TrainRequest
    from kubeml_amd.client import KubemlClient
    srv = _packed_server(tmp_path, 2)
    try:
        c = KubemlClient(srv.url())
        rng = np.random.default_rng(5)
        L = 128
        base = rng.integers(1000, 1100, (16, L))              # a tiny repeating corpus: learnable
        arrs = {"xtr": np.tile(base, (8, 1)).astype(np.int64), "ytr": np.zeros(128, dtype=np.int64),
                "xte": base[:16].astype(np.int64), "yte": np.zeros(16, dtype=np.int64)}
        paths = {}
        for key, v in arrs.items():
            paths[key] = str(tmp_path / f"{key}.npy")
            np.save(paths[key], v)
        c.datasets.create("wiki_tokens", paths["xtr"], paths["ytr"], paths["xte"], paths["yte"])
        c.functions.create("bert", os.path.join(ROOT, "examples", "function_bert.py"))
        jid = c.networks.train(TrainRequest(batch_size=64, epochs=3, dataset="wiki_tokens", lr=3e-4,
                                            function_name="bert",
                                            options=TrainOptions(default_parallelism=2, static_parallelism=True,
                                                                 validate_every=1, k=1, sync="grad")))
        t0 = time.time()
        while c.tasks.status(jid)["state"] == "running":
            assert time.time() - t0 < 600
            time.sleep(0.5)
        st = c.tasks.status(jid)
        assert st["state"] == "finished", (st, c.logs(jid).decode()[-3000:])
        h = c.histories.get(jid).data
        logs = [json.loads(l) for l in c.logs(jid).decode().splitlines() if l.startswith("{")]
        eps = [l for l in logs if l.get("msg") == "epoch finished"]
        assert all(m == "grad-allreduce" for m in h.sync_mode), h.sync_mode
        assert all(len(e["checksums"]) == 2 and _same_model(e) for e in eps), eps
        assert all(np.isfinite(h.train_loss)) and h.train_loss[-1] < h.train_loss[0], h.train_loss
    finally:
        srv.stop()


def test_gpu_worker_killed_mid_round_pool_rebuilds_and_job_finishes(tmp_path):
    """Failure recovery on the GPU data plane: two packed workers (gloo bootstrap, peer-memory
    all-reduce over IPC-mapped HBM), K = 2 K-AVG; rank 1 is killed in epoch 1, round 1 while the
    peers hold each other's IPC mappings.  The job must detect the loss, shut the pool down (the
    survivor's process and its peer mappings go with it), rebuild on the survivor, restore the
    post-init checkpoint and finish every epoch with a history (ml/pkg/train/util.go:144-166)."""
    from kubeml_amd.api.types import TrainOptions, TrainRequest
    from kubeml_amd.client import KubemlClient
    from kubeml_amd.config import Config
    from kubeml_amd.control.server import KubeMLServer
    cfg = Config()
    cfg.store_dir = str(tmp_path / "store")
    cfg.num_gpus = 1
    srv = KubeMLServer(cfg, n_workers=2, use_gpu=True, task_timeout=600,
                       worker_env={"KUBEML_FAULT": "kill:at=round:rank=1:epoch=1:round=1"}).start(
        ports={k_: 0 for k_ in ("controller", "scheduler", "ps", "storage", "metrics")})
    try:
        c = KubemlClient(srv.url())
        arrs = _cifar_like(seed=6)
        paths = {}
        for key, v in arrs.items():
            paths[key] = str(tmp_path / f"{key}.npy")
            np.save(paths[key], v)
        c.datasets.create("cifar10", paths["xtr"], paths["ytr"], paths["xte"], paths["yte"])
        c.functions.create("resnet34", os.path.join(ROOT, "examples", "function_resnet34.py"))
        jid, h, eps = _run_job(c, tmp_path, 2, 2, epochs=2)
        log = c.logs(jid).decode()
        assert "recovering" in log and "epoch failed" in log, log[-3000:]
        assert h.parallelism == [1.0, 1.0], h.parallelism
        assert len(h.train_loss) == 2 and all(np.isfinite(h.train_loss))
        assert len(h.accuracy) == 2
    finally:
        srv.stop()


def test_warm_leaves_a_manual_loop_function_untouched():
    """Job warm-up (KubeModel._warm) on a function written as the reference's manual loop
    (loss.backward(); self.optimizer.step(), like examples/function_lenet.py): its dry train()
    call bypasses self.step and really updates the model, so the warm-up must restore the
    parameters, BN buffers and optimizer state it snapshotted — epoch 1 starts from the
    recovery-base model — and stop scanning train shapes (nothing to capture)."""
    import torch
    import torch.nn as nn
    from kubeml_amd.models.lenet import LeNet
    from kubeml_amd.sdk.dataset import _KubeArgs
    from kubeml_amd.sdk.model import KubeModel

    class _DS:   # the parts of a KubeDataset the warm-up touches
        num_docs, num_val_docs = 4, 0

        def _plan_stream(self, *a, **k):
            return False

        def _load_train_data(self, start, end):
            pass

        def _stream_end(self):
            pass

    class Manual(KubeModel):
        def configure_optimizers(self):
            return torch.optim.SGD(self.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)

        def train(self, batch, batch_index):
            x, y = batch
            self.optimizer.zero_grad()
            loss = nn.functional.cross_entropy(self(x), y)
            loss.backward()
            self.optimizer.step()
            self.calls += 1
            return loss.item()

    torch.manual_seed(0)
    m = Manual(LeNet(), _DS(), gpu=True)
    m.calls = 0
    m.args = _KubeArgs("warmjob", 1, 1, "train", 0, 1, lr=0.1, batch_size=64)
    m.lr, m.batch_size, m.epoch = 0.1, 64, 1
    xs, ys = torch.randn(64, 1, 28, 28), torch.randint(0, 10, (64,))
    m._batches = lambda: iter([(xs, ys), (xs[:32], ys[:32])])
    m._on_train_start()
    c0 = m.model_checksum()
    w0 = [p.detach().clone() for p in m.parameters()]
    assert m._warm() == 0
    assert m.calls == 1                       # the manual loop ran once, then the scan stopped
    assert m.model_checksum() == c0
    assert all(torch.equal(p, q) for p, q in zip(m.parameters(), w0))
    assert len(m.optimizer.state) == 0        # no momentum buffers survive the dry call
