#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k "ride" > gpurun_out/r5/ride_tests2.log 2>&1 || { tail -40 gpurun_out/r5/ride_tests2.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/r5/ride_tests2.log
for r in 1 2 3; do
  for cfg in "0 4f:321 512" "1 4f:321 512" "1 4f:3;3:21 512" "1 4f:3;3:21 1024" "1 4f:32;3:1 512"; do
    set -- $cfg
    tag=$(echo "$1_$2_$3" | tr ':;' '__')
    KUBEML_RIDE=$1 KUBEML_RIDE_PLAN="$2" KUBEML_RIDE_BLOCKS=$3 timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --no-epoch --e2e off > gpurun_out/r5/rs4_${tag}_$r.json 2> gpurun_out/r5/rs4.err || { tail -20 gpurun_out/r5/rs4.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/r5/rs4_${tag}_$r.json').read().strip().splitlines()[-1]);print('ride', '$1', 'plan', '$2', 'blocks', $3, 'rep', $r, d['ms_per_step'])"
  done
done
