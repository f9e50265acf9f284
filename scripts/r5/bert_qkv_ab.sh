#!/bin/bash
# BERT-base: QKV forward on the hand 128x128 tile with the row-pass epilogue (new) vs hipBLASLt (old)
set -o pipefail
out=gpurun_out/r5/bertqkv; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_bert_gpu.py -x -q --timeout 200 --timeout-method thread > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export KUBEML_GEMM_TUNING_FILE=tools/diag/gemm_tuning_r5_pre_qkv.json; else unset KUBEML_GEMM_TUNING_FILE; fi
    timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 3 > $out/bert_${v}_$r.json 2> $out/bert.err || { tail -20 $out/bert.err; exit 1; }
    python -c "import json;d=json.loads(open('$out/bert_${v}_$r.json').read().strip().splitlines()[-1]);print('$v', $r, d['ms_per_step'])" >> $out/ab.txt
  done
done
