#!/bin/bash
# ResNet-34 headline: bench x2 and a kernel timeline at HEAD
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 80 --warmup 5 --no-epoch --e2e off > $out/r34_a$i.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$out/r34_a$i.json'));print('r34', d['ms_per_step'])"
done
rm -rf $out/pr34
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/pr34 -o run -- python bench.py --steps 24 --warmup 5 --no-epoch --e2e off > $out/pr34.log 2>&1 || { tail -20 $out/pr34.log; exit 1; }
db=$(find $out/pr34 -name "*.db" | head -1)
python tools/rocpd_summary.py $db --top 40 > $out/r34_prof.md
python tools/rocpd_timeline.py $db --first-kernel k_augment --nth -2 > $out/r34_timeline.md
rm -rf $out/pr34
tail -1 $out/r34_timeline.md
