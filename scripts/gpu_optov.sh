#!/bin/bash
# Optimizer overlapped with backward: A/B of the side-stream range-SGD grid cap vs off.
set -o pipefail
out=gpurun_out/optov
mkdir -p $out
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-epoch > $out/b_$name.json 2> $out/b_$name.err || { tail -5 $out/b_$name.err; return 1; }
  echo "$name $(python -c "import json;d=json.load(open('$out/b_$name.json'));print(d['ms_per_step'])")"
}
for r in 1 2; do
  run off KUBEML_OPT_OVERLAP=0 || exit 1
  run b16 KUBEML_OPT_OVERLAP=1 KUBEML_OPT_OVERLAP_BLOCKS=16 || exit 1
  run b32 KUBEML_OPT_OVERLAP=1 KUBEML_OPT_OVERLAP_BLOCKS=32 || exit 1
  run b64 KUBEML_OPT_OVERLAP=1 KUBEML_OPT_OVERLAP_BLOCKS=64 || exit 1
  run b128 KUBEML_OPT_OVERLAP=1 KUBEML_OPT_OVERLAP_BLOCKS=128 || exit 1
done
