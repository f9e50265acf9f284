#!/bin/bash
# One-shot backward: numerics, in-graph A/B, engine/model tests.
set -o pipefail
out=gpurun_out/oneshot2
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "oneshot or unroll or bwd_pair or gathered" > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc = 0 ] || exit $rc
for v in 0 1 0 1; do
  KUBEML_BWD_ONESHOT=$v timeout -k 10 200 python bench.py --steps 200 --warmup 10 --e2e off --no-epoch > $out/ab_$v.json 2> $out/ab.err || { tail -5 $out/ab.err; exit 1; }
  echo "bwd_oneshot=$v $(python -c "import json;d=json.load(open('$out/ab_$v.json'));print(d['ms_per_step'], d['loss_first_last'])")"
done
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_models_gpu.py tests/test_determinism_gpu.py -x -q --timeout 200 --timeout-method thread > $out/tests2.log 2>&1
rc=$?; tail -3 $out/tests2.log; exit $rc
