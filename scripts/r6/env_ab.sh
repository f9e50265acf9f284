#!/bin/bash
# round 6: runtime launch knobs around the graphed ResNet-34 step (same box, alternating x2)
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r6/envab
mkdir -p $out
run() {  # name, env assignments...
  local n=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-epoch --e2e off > $out/r34_$n.json 2>$out/r34_$n.err || { tail -5 $out/r34_$n.err; return 1; }
  echo "r34 $n $(tail -1 $out/r34_$n.json | python -c "import json,sys;print(json.loads(sys.stdin.read())['ms_per_step'])")"
}
for rep in 1 2; do
  run base_$rep X=1 || exit 1
  run devkernarg1_$rep HIP_FORCE_DEV_KERNARG=1 || exit 1
  run devkernarg0_$rep HIP_FORCE_DEV_KERNARG=0 || exit 1
  run pktcap0_$rep DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 || exit 1
  run pktcap1_$rep DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 || exit 1
done
