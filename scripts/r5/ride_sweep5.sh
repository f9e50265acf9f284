#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k "ride" > gpurun_out/r5/ride_tests3.log 2>&1 || { tail -40 gpurun_out/r5/ride_tests3.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/r5/ride_tests3.log
for r in 1 2 3; do
  for cfg in "0 conv 512" "1 conv 512" "1 bn 512" "1 bn 256" "1 both 512"; do
    set -- $cfg
    KUBEML_RIDE=$1 KUBEML_RIDE_HOSTKIND=$2 KUBEML_RIDE_BLOCKS=$3 timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --no-epoch --e2e off > gpurun_out/r5/rs5_$1_$2_$3_$r.json 2> gpurun_out/r5/rs5.err || { tail -20 gpurun_out/r5/rs5.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/r5/rs5_$1_$2_$3_$r.json').read().strip().splitlines()[-1]);print('ride', $1, '$2', $3, 'rep', $r, d['ms_per_step'])"
  done
done
