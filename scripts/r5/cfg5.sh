#!/bin/bash
# config 5 through the framework + job warm-up: mask kernel, e2e GPU tests, BERT bench, default bench
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r5
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_transformer_gpu.py tests/test_e2e_gpu.py tests/test_bert_gpu.py -x -v --timeout 300 --timeout-method thread > $out/cfg5_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $out/cfg5_tests.log | tail -30; tail -40 $out/cfg5_tests.log; exit 1; }
grep -E "PASS|FAIL|SKIP" $out/cfg5_tests.log | tail -40
timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 3 > $out/bert_mask.json 2> $out/bert_mask.err || { tail -20 $out/bert_mask.err; exit 1; }
tail -1 $out/bert_mask.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $out/bench_warm.json 2> $out/bench_warm.err || { tail -20 $out/bench_warm.err; exit 1; }
python -c "import json;d=json.loads(open('$out/bench_warm.json').read().strip().splitlines()[-1]);print({k:d.get(k) for k in ('ms_per_step','epoch_time_s','val_images','e2e_epoch_wall_s','e2e_first_epoch_s','e2e_epoch_time_s','e2e_error')})"
