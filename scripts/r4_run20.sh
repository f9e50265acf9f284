#!/bin/bash
# same-box A/B of the ResNet-34 headline: HEAD vs 254f584 (before row-pass / parity / stem changes)
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r4
mkdir -p $out
for i in 1 2; do
( cd ab_old && timeout -k 10 200 python -u bench.py --steps 80 --warmup 5 --no-epoch --e2e off > $out/ab_old_$i.json 2>/dev/null ) || exit 1
python -c "import json;d=json.load(open('$out/ab_old_$i.json'));print('old', d['ms_per_step'])"
timeout -k 10 200 python -u bench.py --steps 80 --warmup 5 --no-epoch --e2e off > $out/ab_new_$i.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$out/ab_new_$i.json'));print('new', d['ms_per_step'])"
done
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "parity or dgrad or conv_bwd_pair" > $out/r20_tests.log 2>&1 || { tail -30 $out/r20_tests.log; exit 1; }
tail -1 $out/r20_tests.log
timeout -k 10 300 python -u tools/bench_resnet50.py > $out/r50_r20.json 2> $out/r50_r20.err || { tail -20 $out/r50_r20.err; exit 1; }
python -c "import json;d=json.load(open('$out/r50_r20.json'));print('r50', d['value'], d['ms_per_step'])"
