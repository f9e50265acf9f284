#!/bin/bash
# Trace at HEAD + A/B of the BN partial-row group reduction threshold.
set -o pipefail
bash scripts/gpu_trace_now.sh || exit 1
out=gpurun_out/grp
mkdir -p $out
for v in 0 256 128 0 256 128; do
  KUBEML_BN_GROUP_MIN=$v timeout -k 10 200 python bench.py --steps 200 --warmup 10 --e2e off --no-epoch > $out/ab_$v.json 2> $out/ab.err || { tail -5 $out/ab.err; exit 1; }
  echo "grp_min=$v $(python -c "import json;d=json.load(open('$out/ab_$v.json'));print(d['ms_per_step'], d['loss_first_last'])")"
done
