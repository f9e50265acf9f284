#!/bin/bash
# attention setprio A/B: ab_old = KML_ATTN_PRIO 0, repo = 1
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r4
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention or attn" > $out/r25_tests.log 2>&1 || { tail -30 $out/r25_tests.log; exit 1; }
tail -1 $out/r25_tests.log
for i in 1 2; do
( cd ab_old && timeout -k 10 120 python tools/attn_micro.py 2>/dev/null | grep -v amdgpu | sed 's/^/prio0 /' ) || exit 1
timeout -k 10 120 python tools/attn_micro.py 2>/dev/null | grep -v amdgpu | sed 's/^/prio1 /' || exit 1
done
