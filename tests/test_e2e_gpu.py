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
