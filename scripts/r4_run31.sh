#!/bin/bash
# same-box A/B: BERT with the plain fwd / dgrad GEMMs on the hand-written kernel vs hipBLASLt
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
for i in 1 2; do
for v in A B C; do
  if [ $v = A ]; then unset KUBEML_GEMM_TUNING_FILE; else export KUBEML_GEMM_TUNING_FILE=scripts/tune_blas_$v.json; fi
  timeout -k 10 300 python -u tools/bench_bert.py > $out/bert_r31_${v}_$i.json 2> $out/bert_r31.err || { tail -20 $out/bert_r31.err; exit 1; }
  python -c "import json;d=json.load(open('$out/bert_r31_${v}_$i.json'));print('$v', d['value'], d['ms_per_step'])"
done
done
unset KUBEML_GEMM_TUNING_FILE
bash scripts/r4_run30.sh
