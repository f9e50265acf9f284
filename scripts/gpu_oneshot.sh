#!/bin/bash
# One-shot panel forward: numerics, isolated A/B, in-graph A/B.
set -o pipefail
out=gpurun_out/oneshot
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "oneshot or unroll or halo or partial_stats" > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python -u tools/halo_micro.py --oneshot > $out/micro.jsonl 2> $out/micro.err || { tail -20 $out/micro.err; exit 1; }
cat $out/micro.jsonl
for v in 0 1 0 1; do
  KUBEML_CONV_ONESHOT=$v timeout -k 10 200 python bench.py --steps 200 --warmup 10 --e2e off --no-epoch > $out/ab_$v.json 2> $out/ab.err || { tail -5 $out/ab.err; exit 1; }
  echo "oneshot=$v $(python -c "import json;d=json.load(open('$out/ab_$v.json'));print(d['ms_per_step'], d['loss_first_last'])")"
done
