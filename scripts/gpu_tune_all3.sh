#!/bin/bash
# In-graph re-tune: forward (table-driven convs) then backward with more candidates.
set -o pipefail
out=gpurun_out/tune4
mkdir -p $out
cp kubeml_amd/ops/conv_tuning.json $out/conv_tuning.json
timeout -k 10 600 python -u tools/tune_ingraph.py --only fwd --topk 4 --out $out/conv_tuning.json > $out/tune_fwd.log 2>&1 || { tail -5 $out/tune_fwd.log; exit 1; }
tail -1 $out/tune_fwd.log
cp $out/conv_tuning.json kubeml_amd/ops/conv_tuning.json
timeout -k 10 900 python -u tools/tune_ingraph.py --only bwd --topk 6 --out $out/conv_tuning.json > $out/tune_bwd.log 2>&1 || { tail -5 $out/tune_bwd.log; exit 1; }
tail -1 $out/tune_bwd.log
