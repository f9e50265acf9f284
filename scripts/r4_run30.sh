#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "kavg" > $out/r30_tests.log 2>&1 || { tail -30 $out/r30_tests.log; exit 1; }
tail -1 $out/r30_tests.log
timeout -k 10 300 python -u tools/bench_resnet50.py --force-comm > $out/r50_sync_comm.json 2> $out/r50_sync.err || { tail -20 $out/r50_sync.err; exit 1; }
python -c "import json;d=json.load(open('$out/r50_sync_comm.json'));print('r50 sync', d['value'], d['ms_per_step'], d.get('comm'), d.get('loss_first_last'))"
timeout -k 10 300 python -u tools/bench_resnet50.py --force-comm --async-kavg > $out/r50_async_comm.json 2> $out/r50_async.err || { tail -20 $out/r50_async.err; exit 1; }
python -c "import json;d=json.load(open('$out/r50_async_comm.json'));print('r50 async', d['value'], d['ms_per_step'], d.get('comm'), d.get('loss_first_last'))"
