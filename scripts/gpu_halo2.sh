#!/bin/bash
# Halo dgrad: numerics, backward split micro, in-graph A/B.
set -o pipefail
out=gpurun_out/halo2
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "halo or conv_fwd_dgrad or bwd_pair or splitk" > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python -u tools/bwd_micro.py > $out/bwd.jsonl 2> $out/bwd.err || { tail -20 $out/bwd.err; exit 1; }
cat $out/bwd.jsonl
for v in 0 1 0 1; do
  KUBEML_DGRAD_HALO=$v timeout -k 10 200 python bench.py --steps 200 --warmup 10 --e2e off --no-epoch > $out/ab_$v.json 2> $out/ab.err || { tail -5 $out/ab.err; exit 1; }
  echo "dgrad_halo=$v $(python -c "import json;d=json.load(open('$out/ab_$v.json'));print(d['ms_per_step'], d['loss_first_last'])")"
done
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_models_gpu.py tests/test_determinism_gpu.py -x -q --timeout 200 --timeout-method thread > $out/tests2.log 2>&1
rc=$?; tail -3 $out/tests2.log; exit $rc
