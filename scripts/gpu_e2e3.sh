#!/bin/bash
# Framework-path epoch with worker traces (graphed validation, HBM-resident split).
set -o pipefail
out=gpurun_out/e2e3
rm -rf $out; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_loader_gpu.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_e2e.py --epochs 4 --validate --trace $out/trace > $out/e2e.json 2> $out/e2e.err || { tail -20 $out/e2e.err; exit 1; }
cut -c1-900 $out/e2e.json
