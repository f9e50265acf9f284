#!/bin/bash
# round 6: BERT step with the 256x256 slab wgrad split counts doubled / x1.5 (in-graph check of the table)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6/wsplit
mkdir -p $out
for rep in 1 2; do
  for v in base x2 x15; do
    f=""; [ $v != base ] && f=$R/tools/diag/gemm_tuning_wgrad_$v.json
    KUBEML_GEMM_TUNING_FILE=$f timeout -k 10 300 python -u tools/bench_bert.py --steps 30 --warmup 5 > $out/b_${v}_$rep.json 2> $out/b_${v}_$rep.err || { tail -20 $out/b_${v}_$rep.err; exit 1; }
    echo "bert $v $rep $(tail -1 $out/b_${v}_$rep.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d.get('ms_per_step'))")"
  done
done
