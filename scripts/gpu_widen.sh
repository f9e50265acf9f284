#!/bin/bash
set -o pipefail
out=gpurun_out/widen
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "bn" > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc = 0 ] || exit $rc
for v in 0 256 128 512 0 256 128 512; do
  KUBEML_BN_ROWS_WIDEN=$v timeout -k 10 200 python bench.py --steps 200 --warmup 10 --e2e off --no-epoch > $out/ab.json 2> $out/ab.err || { tail -5 $out/ab.err; exit 1; }
  echo "widen=$v $(python -c "import json;d=json.load(open('$out/ab.json'));print(d['ms_per_step'], d['loss_first_last'])")"
done
