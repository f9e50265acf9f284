#!/bin/bash
# Refresh the ResNet-34 / ResNet-50 kernel-trace summaries and step timelines at HEAD.
set -o pipefail
out=gpurun_out/final
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run_trace() {  # name first_kernel steps cmd...
  local name=$1 first=$2 steps=$3; shift 3
  rm -rf $out/$name
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name -o run -- "$@" > $out/$name.log 2>&1 || { tail -20 $out/$name.log; return 1; }
  local db=$(find $out/$name -name "*.db" | head -1)
  python tools/rocpd_summary.py $db --steps $steps --top 40 > $out/${name}_summary.md || return 1
  python tools/rocpd_timeline.py $db --first-kernel $first --nth -2 > $out/${name}_timeline.md || return 1
  rm -rf $out/$name
  tail -1 $out/${name}_timeline.md
}
run_trace r34 k_augment 24 python bench.py --steps 20 --warmup 3 --no-epoch || exit 1
run_trace r50 k_augment 10 python tools/bench_resnet50.py --steps 8 --warmup 2 --K 8 || exit 1
timeout -k 10 200 python bench.py > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
cat $out/bench.json
