#!/bin/bash
# CE backward adds the fc bias gradient; unroll gather with 8 chunks per thread: tests + trace + bench.
set -o pipefail
out=gpurun_out/cebias
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_bert_gpu.py -k "ce_ or cross or resnet34 or unrolled or bert" -x -q --timeout 180 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc = 0 ] || exit $rc
bash scripts/gpu_r34_trace.sh || exit 1
grep -n "unroll\|k_ce_\|colsum" gpurun_out/r34t/r34_timeline.md
for r in 1 2; do
timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-epoch > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('r34', d['ms_per_step'])"
done
