"""Synthetic MNIST / CIFAR-10 / CIFAR-100 shaped datasets as .npy files (there is no
network to download the real ones — reference ml/hack/upload_*.sh fetch them), plus an
optional upload to a running server (``kubeml dataset create``).

    python tools/make_datasets.py --out /tmp/ds [--upload] [--learnable]

``--learnable`` plants a class-dependent pattern so accuracy can rise above chance
(used by the end-to-end tests); otherwise images are uniform noise.
"""
import argparse
import os
import subprocess
import sys

import numpy as np

SPECS = {
    "mnist": ((28, 28), 10, 60000, 10000),
    "cifar10": ((32, 32, 3), 10, 50000, 10000),
    "cifar100": ((32, 32, 3), 100, 50000, 10000),
}


def make(name, n_train=None, n_test=None, learnable=False, seed=0):
    shape, classes, ntr, nte = SPECS[name]
    ntr, nte = n_train or ntr, n_test or nte
    rng = np.random.default_rng(seed)
    out = {}
    for split, n in (("train", ntr), ("test", nte)):
        y = rng.integers(0, classes, n).astype(np.int64)
        x = rng.integers(0, 256 if not learnable else 60, (n,) + shape).astype(np.uint8)
        if learnable:
            H, W = shape[0], shape[1]
            for i, k in enumerate(y):
                r = 2 + (k % 4) * (H // 5)
                c = 2 + (k // 4 % 5) * (W // 6)
                x[i, r:r + 4, c:c + 4] = 250
        out[split] = (x, y)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="./datasets")
    ap.add_argument("--names", default="mnist,cifar10")
    ap.add_argument("--train", type=int, default=None)
    ap.add_argument("--test", type=int, default=None)
    ap.add_argument("--learnable", action="store_true")
    ap.add_argument("--upload", action="store_true")
    a = ap.parse_args()
    for name in a.names.split(","):
        d = os.path.join(a.out, name)
        os.makedirs(d, exist_ok=True)
        data = make(name, a.train, a.test, a.learnable)
        files = {}
        for split, (x, y) in data.items():
            files[f"{split}data"] = os.path.join(d, f"x_{split}.npy")
            files[f"{split}labels"] = os.path.join(d, f"y_{split}.npy")
            np.save(files[f"{split}data"], x)
            np.save(files[f"{split}labels"], y)
        print(name, {k: v for k, v in files.items()})
        if a.upload:
            cmd = [sys.executable, "-m", "kubeml_amd.cli", "dataset", "create", "-n", name,
                   "--traindata", files["traindata"], "--trainlabels", files["trainlabels"],
                   "--testdata", files["testdata"], "--testlabels", files["testlabels"]]
            subprocess.run(cmd, check=True)


if __name__ == "__main__":
    main()
