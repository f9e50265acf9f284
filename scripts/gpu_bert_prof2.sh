#!/bin/bash
set -o pipefail
out=gpurun_out
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for mode in 0 1; do
  rm -rf $out/pb$mode
  KUBEML_LINEAR_BLAS=$mode timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/pb$mode -o run -- python tools/bench_bert.py --steps 3 --warmup 1 > $out/pb$mode.log 2>&1 || { tail -20 $out/pb$mode.log; exit 1; }
  db=$(find $out/pb$mode -name "*.db" | head -1)
  python tools/rocpd_summary.py $db --steps 5 --top 30 > $out/bert_prof_blas$mode.md
  rm -rf $out/pb$mode
  head -40 $out/bert_prof_blas$mode.md
done
