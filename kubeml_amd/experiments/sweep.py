"""Grid sweeps over (batch, K, parallelism) — reference ml/experiments/train.py and
common/utils.py:12-28 (grids), 54-80 (resume: skip experiments already saved).

    python -m kubeml_amd.experiments.sweep --network lenet --out results/ [--dry]
"""
from __future__ import annotations

import argparse
import itertools
import os

from ..api.types import TrainOptions, TrainRequest
from .experiment import KubemlExperiment, get_hash, get_title

GRIDS = {
    "lenet": {"batch": [128, 64, 32, 16], "k": [-1, 32, 16, 8], "parallelism": [1, 2, 4, 8],
              "dataset": "mnist", "function": "lenet", "lr": 0.01},
    "resnet34": {"batch": [256, 128, 64, 32], "k": [-1, 32, 16, 8], "parallelism": [2, 4, 8],
                 "dataset": "cifar10", "function": "resnet34", "lr": 0.1},
}


def requests_for(network: str, epochs: int, grid: dict = None):
    g = grid or GRIDS[network]
    for b, k, p in itertools.product(g["batch"], g["k"], g["parallelism"]):
        yield TrainRequest(model_type=network, batch_size=b, epochs=epochs, dataset=g["dataset"], lr=g["lr"],
                           function_name=g["function"],
                           options=TrainOptions(default_parallelism=p, static_parallelism=True, k=k,
                                                validate_every=1, goal_accuracy=100))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--network", choices=sorted(GRIDS), default="lenet")
    ap.add_argument("--epochs", type=int, default=30)
    ap.add_argument("--out", default="./results")
    ap.add_argument("--url", default=None)
    ap.add_argument("--replications", type=int, default=1)
    ap.add_argument("--dry", action="store_true")
    a = ap.parse_args(argv)
    done = set()
    if os.path.isdir(a.out):
        import json
        for f in os.listdir(a.out):
            if f.endswith(".json"):
                with open(os.path.join(a.out, f)) as fh:
                    done.add(json.load(fh).get("hash"))
    for req in requests_for(a.network, a.epochs):
        title = get_title(req)
        if get_hash(title) in done:
            print("skip", title)
            continue
        for _ in range(a.replications):
            print("run", title)
            if a.dry:
                continue
            e = KubemlExperiment(title, req, url=a.url)
            e.run()
            print("saved", e.save(a.out))


if __name__ == "__main__":
    main()
