#!/bin/bash
# same-box A/B: FFN2 dgrad with the GELU-backward epilogue (shipped, E) vs hipBLASLt dgrad +
# the separate GELU-backward / bias column-sum pass (F)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
for i in 1 2; do
for v in E F; do
  if [ $v = E ]; then unset KUBEML_GEMM_TUNING_FILE; else export KUBEML_GEMM_TUNING_FILE=scripts/tune_blas_F.json; fi
  timeout -k 10 300 python -u tools/bench_bert.py > $out/bert_r42_${v}_$i.json 2> $out/bert_r42.err || { tail -20 $out/bert_r42.err; exit 1; }
  echo "$v $(tail -1 $out/bert_r42_${v}_$i.json | cut -c60-130)"
done
done
