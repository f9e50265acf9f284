#!/bin/bash
# A/B: dgrad plan of the ungrouped 1x1 convs (their wgrad runs on the slab GEMM)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
for v in base 128,64,64,1,1 64,128,64,1,1 128,128,32,1,0 128,128,64,1,1 base; do
  if [ $v = base ]; then unset KUBEML_AB_DGRAD1X1; else export KUBEML_AB_DGRAD1X1=$v; fi
  timeout -k 10 300 python -u tools/bench_resnet50.py > $out/r50_r41.json 2> $out/r50_r41.err || { echo "$v FAILED"; tail -5 $out/r50_r41.err; continue; }
  echo "$v $(tail -1 $out/r50_r41.json | cut -c100-175)"
done
