"""Experiment harness + analysis (reference ml/experiments): TTA definitions, best
combinations, the online K predictor, and a KubemlExperiment run through the CLI
against a live CPU server."""
import math
import os

import numpy as np

from kubeml_amd.experiments.analysis import KOptimizer, best_combinations, summarize, tta, tta_crossbow


def test_tta_definitions():
    row = {"accuracy": [10, 50, 71, 69, 72, 73, 75], "epoch_duration": [1, 2, 3, 4, 5, 6, 7]}
    assert tta(70, row) == 3
    assert tta_crossbow(70, row) == 6      # median(71,69,72,73,75)... first window with median>=70 ends at idx 5
    assert math.isnan(tta(99, row))
    assert math.isnan(tta_crossbow(99, row))
    s = summarize({"accuracy": [1, 2], "epoch_duration": [3, 9], "parallelism": [4, 4], "k": -1, "batch_size": 32})
    assert s["k"] == math.inf and s["global_batch"] == 128 and s["time"] == 9


def test_best_combinations():
    rows = [{"batch_size": 32, "tta": 5.0, "k": 8}, {"batch_size": 32, "tta": 3.0, "k": 16},
            {"batch_size": 64, "tta": 7.0, "k": 8}, {"batch_size": 64, "tta": math.nan, "k": 16}]
    b = best_combinations(rows, "tta")
    assert [(r["batch_size"], r["k"]) for r in b] == [(32, 16), (64, 8)]


def test_k_optimizer_online():
    rng = np.random.default_rng(0)
    X = np.array([[b, 0.01, p, k] for b in (32, 64, 128) for p in (1, 2, 4) for k in (2, 8, 16, 64)], dtype=float)
    y_time = 1000.0 / (X[:, 3] + 1) + X[:, 0] * 0.1 + rng.normal(0, 1, len(X))
    y_acc = 90 - 0.05 * X[:, 3] + rng.normal(0, 0.1, len(X))
    ko = KOptimizer(X, y_acc, y_time)
    preds = ko.predict(64, 0.01, 2)
    assert [p["k"] for p in preds] == KOptimizer.Ks
    k = ko.best_k(64, 0.01, 2)
    assert k in KOptimizer.Ks
    ko.update([64, 0.01, 2, 16], 50.0, 88.0)


def test_kubeml_experiment_via_cli(tmp_path):
    from kubeml_amd.api.types import TrainOptions, TrainRequest
    from kubeml_amd.client import KubemlClient
    from kubeml_amd.config import Config
    from kubeml_amd.control.server import KubeMLServer
    from kubeml_amd.experiments.experiment import KubemlExperiment, get_title
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import make_datasets
    cfg = Config()
    cfg.store_dir = str(tmp_path / "store")
    srv = KubeMLServer(cfg, n_workers=1, use_gpu=False, task_timeout=300).start(
        ports={k: 0 for k in ("controller", "scheduler", "ps", "storage", "metrics")})
    try:
        c = KubemlClient(srv.url())
        d = make_datasets.make("mnist", 640, 128, learnable=True)
        paths = {}
        for split, (x, y) in d.items():
            paths[split] = (str(tmp_path / f"x{split}.npy"), str(tmp_path / f"y{split}.npy"))
            np.save(paths[split][0], x)
            np.save(paths[split][1], y)
        c.datasets.create("mnist", paths["train"][0], paths["train"][1], paths["test"][0], paths["test"][1])
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        c.functions.create("lenet", os.path.join(root, "examples", "function_lenet.py"))
        req = TrainRequest(model_type="lenet", batch_size=64, epochs=2, dataset="mnist", lr=0.05,
                           function_name="lenet",
                           options=TrainOptions(default_parallelism=1, static_parallelism=True, k=-1,
                                                validate_every=1))
        e = KubemlExperiment(get_title(req), req, url=srv.url(), use_cli=True, poll_s=0.3)
        h = e.run()
        assert len(h.data.train_loss) == 2
        p = e.save(str(tmp_path / "res"))
        from kubeml_amd.experiments.analysis import load_rows
        rows = load_rows(str(tmp_path / "res"))
        assert rows[0]["id"] == e.network_id and rows[0]["batch_size"] == 64 and len(rows[0]["accuracy"]) == 2
    finally:
        srv.stop()
