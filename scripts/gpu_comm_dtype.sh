#!/bin/bash
# Single-rank RCCL rehearsal of the gradient all-reduce (force-comm, graph-captured) in fp32
# and bf16-compressed form; engine GPU tests.
set -o pipefail
out=gpurun_out/comm
mkdir -p $out
for d in fp32 bf16; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-epoch --force-comm --overlap on --comm-dtype $d > $out/$d.json 2> $out/$d.err || { tail -20 $out/$d.err; exit 1; }
  python -c "import json;d=json.loads(open('$out/$d.json').read().strip().splitlines()[-1]);print('$d', d['ms_per_step'], d['loss_first_last'], d['config']['grad_comm_dtype'])"
done
