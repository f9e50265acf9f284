#!/bin/bash
# failure-path + multirank GPU tests, e2e warm-up check
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r5
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_multirank_gpu.py tests/test_e2e_gpu.py tests/test_peer_gpu.py -x -v --timeout 300 --timeout-method thread > $out/faults_tests.log 2>&1 || { grep -E "PASS|FAIL|Error" $out/faults_tests.log | tail -30; tail -50 $out/faults_tests.log; exit 1; }
grep -E "PASS|FAIL|SKIP" $out/faults_tests.log | tail -40
