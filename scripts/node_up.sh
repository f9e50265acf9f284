#!/usr/bin/env bash
# Bring up KubeML on this node (reference: ml/hack/cluster_config.sh installs fission,
# prometheus and the helm chart).  Usage: scripts/node_up.sh [store_dir]
set -euo pipefail
cd "$(dirname "$0")/.."
export KUBEML_STORE_DIR="${1:-${KUBEML_STORE_DIR:-$HOME/.kubeml}}"
python -m kubeml_amd._build
exec python -m kubeml_amd.control.server
