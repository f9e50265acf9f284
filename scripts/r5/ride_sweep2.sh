#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r5
for r in 1 2 3; do
  for cfg in "0 128" "1 512" "1 1024" "1 2048"; do
    set -- $cfg
    KUBEML_RIDE=$1 KUBEML_RIDE_BLOCKS=$2 timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --no-epoch --e2e off > gpurun_out/r5/rs2_$1_$2_$r.json 2> gpurun_out/r5/rs2_$1_$2_$r.err || { tail -20 gpurun_out/r5/rs2_$1_$2_$r.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/r5/rs2_$1_$2_$r.json').read().strip().splitlines()[-1]);print('ride', $1, 'blocks', $2, 'rep', $r, d['ms_per_step'])"
  done
done
