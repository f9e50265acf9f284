#!/bin/bash
# BN counters bumped by the fused stem kernel: engine/model tests + bench + trace.
set -o pipefail
out=gpurun_out/counters
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_models_gpu.py tests/test_kernels_gpu.py -k "graphed or stem or maxpool or resnet or vgg" -x -q --timeout 180 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc = 0 ] || exit $rc
bash scripts/gpu_r34_trace.sh || exit 1
grep -c "add_i64" gpurun_out/r34t/r34_timeline.md || true
for r in 1 2; do
timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-epoch > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('r34', d['ms_per_step'])"
done
