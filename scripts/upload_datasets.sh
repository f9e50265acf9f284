#!/usr/bin/env bash
# Create MNIST / CIFAR-10 / CIFAR-100 shaped datasets and upload them (reference
# ml/hack/upload_{mnist,cifar10,cifar100}.sh download the real ones; this box has no
# network, so the data is synthetic with the real shapes).
set -euo pipefail
cd "$(dirname "$0")/.."
python tools/make_datasets.py --out "${1:-/tmp/kubeml-datasets}" --names mnist,cifar10,cifar100 --upload
