#!/bin/bash
# config 5: framework BERT step (kubeml train, K=1 grad-sync, 1 worker) vs tools/bench_bert.py, same box
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 3 > gpurun_out/r5/bert_bench_ab.json 2> gpurun_out/r5/bert_bench_ab.err || { tail -20 gpurun_out/r5/bert_bench_ab.err; exit 1; }
ms=$(python -c "import json;print(json.loads(open('gpurun_out/r5/bert_bench_ab.json').read().strip().splitlines()[-1])['ms_per_step'])")
echo "bench_bert ms/step $ms"
timeout -k 10 600 python -u tools/bench_bert_e2e.py --steps 24 --epochs 4 --bench-ms $ms > gpurun_out/r5/bert_e2e.json 2> gpurun_out/r5/bert_e2e.err || { tail -30 gpurun_out/r5/bert_e2e.err; exit 1; }
tail -1 gpurun_out/r5/bert_e2e.json
