#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r5
for r in 1 2 3; do
  for cfg in "0 3 128" "1 3 1024" "1 32 512" "1 32 1024" "1 321 512" "1 321 1024"; do
    set -- $cfg
    KUBEML_RIDE=$1 KUBEML_RIDE_HOSTS=$2 KUBEML_RIDE_BLOCKS=$3 timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --no-epoch --e2e off > gpurun_out/r5/rs3_$1_$2_$3_$r.json 2> gpurun_out/r5/rs3.err || { tail -20 gpurun_out/r5/rs3.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/r5/rs3_$1_$2_$3_$r.json').read().strip().splitlines()[-1]);print('ride', $1, 'hosts', '$2', 'blocks', $3, 'rep', $r, d['ms_per_step'])"
  done
done
