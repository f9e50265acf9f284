#!/bin/bash
# round 6: final-row BN statistics + BN-backward fold — numerics, then alternating A/B
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r6/ab_final
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bnb_gpu.py \
  "tests/test_kernels_gpu.py::test_dgrad_final_row_matches_fp32" "tests/test_kernels_gpu.py::test_dgrad_emits_consumer_bn_partials" \
  "tests/test_kernels_gpu.py::test_conv_bwd_pair_matches_separate" "tests/test_kernels_gpu.py::test_grouped_partial_rows" \
  "tests/test_kernels_gpu.py::test_unrolled_conv_bwd_matches_3x3" "tests/test_kernels_gpu.py::test_conv_halo_dgrad" \
  tests/test_models_gpu.py > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for rep in 1 2; do
  for v in "0 0" "1 0" "1 1"; do
    set -- $v
    KUBEML_FINAL_ROWS=$1 KUBEML_BNB_FOLD=$2 timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-epoch --e2e off > $out/b_$1$2_$rep.json 2> $out/b_$1$2_$rep.err || { tail -20 $out/b_$1$2_$rep.err; exit 1; }
    echo "final=$1 bnb=$2 rep=$rep $(python -c "import json,sys;d=json.loads(open('$out/b_$1$2_$rep.json').read().strip().splitlines()[-1]);print(d['ms_per_step'])")"
  done
done
