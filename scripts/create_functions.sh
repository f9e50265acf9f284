#!/usr/bin/env bash
# Register the example functions (reference ml/hack/create_functions.sh).
set -euo pipefail
cd "$(dirname "$0")/.."
for f in lenet resnet34 resnet32 vgg16; do
  [ -f "examples/function_${f}.py" ] && python -m kubeml_amd.cli fn create --name "$f" --code "examples/function_${f}.py" || true
done
python -m kubeml_amd.cli fn list
