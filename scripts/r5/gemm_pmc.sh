#!/bin/bash
# L2 behaviour of the hand 256x256 phase tile vs hipBLASLt on BERT's QKV dgrad / FFN2 fwd shapes
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r5/gemm_pmc
mkdir -p $out
run() {  # name, counters, args...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc $ctr -d $out/$name -o run -- python3 $R/tools/gemm_one.py "$@" > $out/$name.log 2>&1 || { echo "pmc $name failed"; tail -5 $out/$name.log; return 1; }
}
for shp in "1 16384 768 2304" "0 16384 768 3072"; do
  set -- $shp
  tag=l$1_n$3_k$4
  run hand_hit_$tag "TCC_HIT_sum TCC_MISS_sum" --layout $1 --M $2 --N $3 --K $4 --tile 256,256,8 --reps 10 || exit 1
  run blas_hit_$tag "TCC_HIT_sum TCC_MISS_sum" --layout $1 --M $2 --N $3 --K $4 --torch --reps 10 || exit 1
  run hand_ea_$tag "TCC_EA0_RDREQ_sum" --layout $1 --M $2 --N $3 --K $4 --tile 256,256,8 --reps 10 || exit 1
  run blas_ea_$tag "TCC_EA0_RDREQ_sum" --layout $1 --M $2 --N $3 --K $4 --torch --reps 10 || exit 1
done
for f in $(find $out -name "*counter_collection.csv"); do echo "== $f"; python3 $R/tools/pmc_summary.py $f | head -8; done
