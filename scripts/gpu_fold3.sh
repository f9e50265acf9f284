#!/bin/bash
set -o pipefail
out=gpurun_out/fold3
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread -k "bnin or bn_fold or oneshot or unroll or resnet or halo" > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc = 0 ] || exit $rc
for v in 1 0 1 0; do
  KUBEML_BN_FOLD=$v timeout -k 10 200 python bench.py --steps 200 --warmup 10 --e2e off --no-epoch > $out/ab.json 2> $out/ab.err || { tail -5 $out/ab.err; exit 1; }
  echo "fold=$v $(python -c "import json;d=json.load(open('$out/ab.json'));print(d['ms_per_step'], d['loss_first_last'])")"
done
