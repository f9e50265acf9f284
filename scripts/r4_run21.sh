#!/bin/bash
# same-box per-kernel timelines of the R34 step: HEAD vs 254f584
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r4
mkdir -p $out
rm -rf $out/pab_old $out/pab_new
( cd ab_old && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/pab_old -o run -- python bench.py --steps 24 --warmup 5 --no-epoch --e2e off > $out/pab_old.log 2>&1 ) || { tail -20 $out/pab_old.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/pab_new -o run -- python bench.py --steps 24 --warmup 5 --no-epoch --e2e off > $out/pab_new.log 2>&1 || { tail -20 $out/pab_new.log; exit 1; }
for v in old new; do
db=$(find $out/pab_$v -name "*.db" | head -1)
python tools/rocpd_summary.py $db --top 40 > $out/ab_${v}_prof.md
python tools/rocpd_timeline.py $db --first-kernel k_augment --nth -3 > $out/ab_${v}_timeline.md
tail -1 $out/ab_${v}_timeline.md
done
rm -rf $out/pab_old $out/pab_new
