#!/bin/bash
# same-box A/B: BERT GEMM routing variants (C: plain fwd/dgrad on hipBLASLt; D: + FFN1 fwd as
# library GEMM + GELU pass; E: + MLM-head GEMMs), then the K-AVG kernel test
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
for i in 1 2; do
for v in C D E; do
  export KUBEML_GEMM_TUNING_FILE=scripts/tune_blas_$v.json
  timeout -k 10 300 python -u tools/bench_bert.py > $out/bert_r32_${v}_$i.json 2> $out/bert_r32.err || { tail -20 $out/bert_r32.err; exit 1; }
  python -c "import json;d=json.load(open('$out/bert_r32_${v}_$i.json'));print('$v', d['value'], d['ms_per_step'])"
done
done
unset KUBEML_GEMM_TUNING_FILE
bash scripts/r4_run30.sh
