#!/bin/bash
# Does a multi-stream graph cost by itself? One empty side-stream branch per step vs none;
# and the one-line JSON contract with RCCL initialised (force-comm rehearsal).
set -o pipefail
out=gpurun_out/fork
mkdir -p $out
for r in 1 2; do
  for v in 0 1; do
    KUBEML_OPT_OVERLAP=0 KUBEML_DEBUG_FORK=$v timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-epoch > $out/b_$v.json 2> $out/b_$v.err || { tail -5 $out/b_$v.err; exit 1; }
    echo "debug_fork=$v $(python -c "import json;d=json.load(open('$out/b_$v.json'));print(d['ms_per_step'])")"
  done
done
KUBEML_OPT_OVERLAP=0 timeout -k 10 200 python bench.py --force-comm --steps 100 --no-epoch > $out/fc.json 2> $out/fc.err || { tail -5 $out/fc.err; exit 1; }
echo "force-comm stdout lines: $(wc -l < $out/fc.json)"
python -c "import json;d=json.load(open('$out/fc.json'));print('force-comm', d['ms_per_step'], d.get('ranks_in_sync'), d['config']['graph_comm'])"
