#!/bin/bash
# round 6: stem-wgrad SGD rider (4f:321;123:s) vs the round-5 plan (4f:321), alternating, + tests
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r6/ab_ride
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py \
  tests/test_models_gpu.py tests/test_e2e_gpu.py::test_warm_leaves_a_manual_loop_function_untouched \
  "tests/test_kernels_gpu.py::test_conv_bwd_pair_matches_separate" > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for rep in 1 2; do
  for plan in "4f:321" "4f:321;123:s"; do
    tag=$(echo $plan | tr ':;' '__')
    KUBEML_RIDE_PLAN="$plan" timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-epoch --e2e off > $out/b_${tag}_$rep.json 2> $out/b_${tag}_$rep.err || { tail -20 $out/b_${tag}_$rep.err; exit 1; }
    echo "plan=$plan rep=$rep $(python -c "import json;d=json.loads(open('$out/b_${tag}_$rep.json').read().strip().splitlines()[-1]);print(d['ms_per_step'])")"
  done
done
bash scripts/r6/tl.sh tl_ride
