#!/bin/bash
# Kernel-trace profile of the headline step (rocprofv3) -> per-kernel summary + timeline.
set -o pipefail
out=gpurun_out/r3prof
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run_trace() {  # name first_kernel steps cmd...
  local name=$1 first=$2 steps=$3; shift 3
  rm -rf $out/$name
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name -o run -- "$@" > $out/$name.log 2>&1 || { tail -20 $out/$name.log; return 1; }
  local db=$(find $out/$name -name "*.db" | head -1)
  python tools/rocpd_summary.py $db --steps $steps --top 45 > $out/${name}_summary.md || return 1
  python tools/rocpd_timeline.py $db --first-kernel $first --nth -2 > $out/${name}_timeline.md || return 1
  rm -rf $out/$name
  tail -1 $out/${name}_timeline.md
}
run_trace r34 k_augment 24 python bench.py --steps 20 --warmup 3 --no-epoch || exit 1
KUBEML_FULL_ZERO=1 run_trace r34_fullzero k_augment 24 python bench.py --steps 20 --warmup 3 --no-epoch || exit 1
head -60 $out/r34_summary.md
