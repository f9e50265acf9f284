#!/bin/bash
set -o pipefail
out=gpurun_out
mkdir -p $out
for i in 1 2 3; do
timeout -k 10 200 python -u -m pytest tests/test_engine_gpu.py -q --timeout 150 --timeout-method thread -k "one_update_per_batch" > $out/eng_$i.log 2>&1
tail -1 $out/eng_$i.log; grep "AssertionError: (" $out/eng_$i.log | cut -c1-200
done
