#!/bin/bash
# rider block-count sweep (bench, 100 steps) + per-dispatch timeline with the rider on
set -o pipefail
mkdir -p gpurun_out/r5
for r in 1 2; do
  for cfg in "0 128" "1 32" "1 64" "1 256" "1 512"; do
    set -- $cfg
    KUBEML_RIDE=$1 KUBEML_RIDE_BLOCKS=$2 timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-epoch --e2e off > gpurun_out/r5/rs_$1_$2_$r.json 2> gpurun_out/r5/rs_$1_$2_$r.err || { tail -20 gpurun_out/r5/rs_$1_$2_$r.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/r5/rs_$1_$2_$r.json').read().strip().splitlines()[-1]);print('ride', $1, 'blocks', $2, 'rep', $r, d['ms_per_step'])"
  done
done
cd /tmp && cd $GRAFT_REPO_ROOT
out=$GRAFT_REPO_ROOT/gpurun_out/r5
rm -rf $out/prof_ride
KUBEML_RIDE=1 KUBEML_RIDE_BLOCKS=64 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_ride -o run -- python bench.py --steps 20 --warmup 3 --no-epoch --e2e off > $out/prof_ride.log 2>&1 || { tail -20 $out/prof_ride.log; exit 1; }
db=$(find $out/prof_ride -name "*.db" | head -1)
python tools/rocpd_timeline.py $db --first-kernel k_augment --nth -2 > $out/r34_timeline_ride.md
tail -3 $out/r34_timeline_ride.md
rm -rf $out/prof_ride
