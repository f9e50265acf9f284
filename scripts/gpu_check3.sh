#!/bin/bash
# Focused GPU suite after the round-3 kernel work.
set -o pipefail
out=gpurun_out/check3
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_engine_gpu.py tests/test_determinism_gpu.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; exit $rc
