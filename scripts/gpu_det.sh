#!/bin/bash
set -o pipefail
out=gpurun_out
mkdir -p $out
for cfg in "RUNS=10" "RUNS=10 KUBEML_CONV_NOSPLIT=1" "RUNS=10 KUBEML_BN_FUSE=0" "RUNS=10 KUBEML_CONV_NOSPLIT_W=1"; do
  echo "== $cfg"
  env $cfg timeout -k 10 200 python tools/determinism_check.py > $out/det.log 2>&1 || { tail -5 $out/det.log; exit 1; }
  grep "^run" $out/det.log | awk '{print $1,$2,$3,$7,$8,$10}'
done
