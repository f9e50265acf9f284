#!/bin/bash
# R50 with the swept 1x1 wgrad table (shipped) vs the first table (scripts/wgrad_gemm_r50_v1.json);
# then the extended-splits sweep on the 128x128 tile
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
for i in 1 2; do
  unset KUBEML_WGRAD_GEMM_FILE
  timeout -k 10 300 python -u tools/bench_resnet50.py > $out/r50_r38_S_$i.json 2> $out/r50_r38.err || { tail -20 $out/r50_r38.err; exit 1; }
  echo "S $(tail -1 $out/r50_r38_S_$i.json | cut -c1-160)"
  export KUBEML_WGRAD_GEMM_FILE=scripts/wgrad_gemm_r50_v1.json
  timeout -k 10 300 python -u tools/bench_resnet50.py > $out/r50_r38_V_$i.json 2> $out/r50_r38.err || { tail -20 $out/r50_r38.err; exit 1; }
  echo "V $(tail -1 $out/r50_r38_V_$i.json | cut -c1-160)"
done
unset KUBEML_WGRAD_GEMM_FILE
timeout -k 10 600 python -u tools/wgrad_1x1.py --sweep --tiles > $out/wgrad_1x1_sweep2.jsonl 2> $out/wgrad_sweep.err || { tail -20 $out/wgrad_sweep.err; exit 1; }
python -c "
import json
for l in open('$out/wgrad_1x1_sweep2.jsonl'):
    d=json.loads(l); print(d['P'],d['Cout'],d['Cin'],'conv',d['conv_us'],'best',d['best'],d['best_us'])
"
