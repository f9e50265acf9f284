#!/bin/bash
# VGG-16 / Adam: per-stage optimizer overlap (classifier update beside the conv backward) A/B
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k "overlap" > gpurun_out/r5/vgg_ov_tests.log 2>&1 || { tail -30 gpurun_out/r5/vgg_ov_tests.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/r5/vgg_ov_tests.log
for r in 1 2; do
  for ov in off on; do
    timeout -k 10 300 python -u tools/bench_vgg.py --steps 50 --warmup 5 --opt-overlap $ov > gpurun_out/r5/vgg_ov_${ov}_$r.json 2> gpurun_out/r5/vgg_ov_${ov}_$r.err || { tail -20 gpurun_out/r5/vgg_ov_${ov}_$r.err; exit 1; }
    tail -1 gpurun_out/r5/vgg_ov_${ov}_$r.json | cut -c1-260
  done
done
