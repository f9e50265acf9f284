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
