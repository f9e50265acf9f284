#!/bin/bash
# SGD rider: exactness tests, then bench A/B (KUBEML_RIDE 0/1, two alternating reps)
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k "ride or overlap or graphed_step" > gpurun_out/r5/ride_tests.log 2>&1 || { tail -40 gpurun_out/r5/ride_tests.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/r5/ride_tests.log
for r in 1 2; do
  for rd in 0 1; do
    KUBEML_RIDE=$rd timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-epoch --e2e off > gpurun_out/r5/ride_${rd}_$r.json 2> gpurun_out/r5/ride_${rd}_$r.err || { tail -20 gpurun_out/r5/ride_${rd}_$r.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/r5/ride_${rd}_$r.json').read().strip().splitlines()[-1]);print('ride', $rd, 'rep', $r, d['ms_per_step'], d['loss_first_last'])"
  done
done
