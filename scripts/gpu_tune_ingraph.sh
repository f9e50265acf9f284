#!/bin/bash
# In-graph conv plan tuning of the headline step (tools/tune_ingraph.py), then the bench.
set -o pipefail
out=gpurun_out/ig
mkdir -p $out
timeout -k 10 1000 python -u tools/tune_ingraph.py --out $out/conv_tuning.json --steps 100 --topk ${TOPK:-3} --only ${ONLY:-fwd,bwd} > $out/tune.log 2>&1 || { tail -20 $out/tune.log; exit 1; }
grep -E "chosen|start_ms|final_ms" $out/tune.log
cp $out/conv_tuning.json kubeml_amd/ops/conv_tuning.json
timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-epoch > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
cat $out/bench.json
