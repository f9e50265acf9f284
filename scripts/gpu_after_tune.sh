#!/bin/bash
set -o pipefail
out=gpurun_out/aftertune
mkdir -p $out
timeout -k 10 200 python -u tools/stem_wgrad_sweep.py > $out/stem_wgrad.json 2> $out/stem.err || { tail -5 $out/stem.err; exit 1; }
python -c "import json;d=json.load(open('$out/stem_wgrad.json'));print(d['current'], d['best5'])"
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 --e2e off --no-epoch > $out/ab.json 2> $out/ab.err || { tail -5 $out/ab.err; exit 1; }
  echo "bench $(python -c "import json;d=json.load(open('$out/ab.json'));print(d['ms_per_step'], d['loss_first_last'])")"
done
