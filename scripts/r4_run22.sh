#!/bin/bash
# kernarg experiment: ab_old = HEAD with 512 untouched bytes appended to ConvArgs
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r4
mkdir -p $out
for i in 1 2 3; do
( cd ab_old && timeout -k 10 200 python -u bench.py --steps 80 --warmup 5 --no-epoch --e2e off > $out/ab_pad_$i.json 2>/dev/null ) || exit 1
python -c "import json;d=json.load(open('$out/ab_pad_$i.json'));print('pad', d['ms_per_step'])"
timeout -k 10 200 python -u bench.py --steps 80 --warmup 5 --no-epoch --e2e off > $out/ab_head_$i.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$out/ab_head_$i.json'));print('head', d['ms_per_step'])"
done
