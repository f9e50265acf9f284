#!/bin/bash
# Loader test, then the end-to-end framework bench (kubeml train through the server) on
# 1 GPU, with and without per-epoch validation, next to bench.py's step rate.
set -o pipefail
out=gpurun_out
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_loader_gpu.py -x -v --timeout 120 --timeout-method thread > $out/loader_tests.log 2>&1
rc=$?; tail -4 $out/loader_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python bench.py > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
img=$(python -c "import json;print(json.load(open('$out/bench.json'))['value'])")
cat $out/bench.json
timeout -k 10 400 python tools/bench_e2e.py --epochs 4 --bench-img-s $img > $out/e2e.json 2> $out/e2e.err || { tail -20 $out/e2e.err; exit 1; }
cat $out/e2e.json
timeout -k 10 400 python tools/bench_e2e.py --epochs 3 --validate --bench-img-s $img > $out/e2e_val.json 2> $out/e2e_val.err || { tail -20 $out/e2e_val.err; exit 1; }
cat $out/e2e_val.json
