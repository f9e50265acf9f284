#!/bin/bash
# Stem halo kernel: numerics + in-graph A/B; then trace at HEAD and the BN row-grouping A/B.
set -o pipefail
out=gpurun_out/stem
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread -k "stem or resnet or bn_relu_maxpool" > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc = 0 ] || exit $rc
for v in 0 1 0 1; do
  KUBEML_CONV_STEM=$v timeout -k 10 200 python bench.py --steps 200 --warmup 10 --e2e off --no-epoch > $out/ab_$v.json 2> $out/ab.err || { tail -5 $out/ab.err; exit 1; }
  echo "stem=$v $(python -c "import json;d=json.load(open('$out/ab_$v.json'));print(d['ms_per_step'], d['loss_first_last'])")"
done
bash scripts/gpu_grp.sh
