#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
timeout -k 10 600 python -u tools/wgrad_1x1.py --sweep > $out/wgrad_1x1_sweep.jsonl 2> $out/wgrad_sweep.err || { tail -20 $out/wgrad_sweep.err; exit 1; }
python -c "
import json
for l in open('$out/wgrad_1x1_sweep.jsonl'):
    d=json.loads(l); print(d['P'],d['Cout'],d['Cin'],'conv',d['conv_us'],'best',d['best'],d['best_us'])
"
