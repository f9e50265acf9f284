#!/bin/bash
# attention: cheaper dropout words in the forward, vectorised dKV LDS reads; shard rehearsal
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention or attn" > $out/attn_tests.log 2>&1 || { tail -30 $out/attn_tests.log; exit 1; }
tail -1 $out/attn_tests.log
for i in 1 2; do
timeout -k 10 120 python tools/attn_micro.py > $out/attn_micro_$i.jsonl 2>&1 || { cat $out/attn_micro_$i.jsonl; exit 1; }
grep -v amdgpu.ids $out/attn_micro_$i.jsonl
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $out/attn_prof -o attn -- python tools/attn_micro.py > $out/attn_prof.log 2>&1 || { tail -20 $out/attn_prof.log; exit 1; }
bash scripts/r4_run10.sh
