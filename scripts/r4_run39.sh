#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_determinism_gpu.py -x -q --timeout 200 --timeout-method thread > $out/r39_det.log 2>&1 || { grep -n "^E \|rc = \|Error" $out/r39_det.log | head -20; exit 1; }
tail -1 $out/r39_det.log
bash scripts/r4_full.sh
