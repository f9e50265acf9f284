#!/bin/bash
# Data-counter advance folded into the SGD launch: tests, then A/B on one box (1 = folded, 0 = k_advance).
set -o pipefail
out=gpurun_out/advopt
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_models_gpu.py -k "sgd or graphed or counter or bench" -x -q --timeout 180 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc = 0 ] || exit $rc
for r in 1 2 3; do
for v in 1 0; do
KUBEML_ADV_IN_OPT=$v timeout -k 10 200 python bench.py --steps 300 --warmup 10 > $out/bench$v.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench$v.json'));print('adv_in_opt=$v', d['ms_per_step'], d['epoch_time_s'], d['loss_first_last'])"
done
done
