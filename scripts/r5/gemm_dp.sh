#!/bin/bash
# k_gemm8 DMA issue position A/B (KUBEML_GEMM8_DP 0..3): numerics then BERT fwd/dgrad shapes
set -o pipefail
mkdir -p gpurun_out/r5
SH="0:16384:2304:768;1:16384:768:2304;0:16384:768:768;1:16384:768:768;0:16384:3072:768;1:16384:768:3072;0:16384:768:3072;1:16384:3072:768"
for dp in 1 2 3; do
  KUBEML_GEMM8_DP=$dp timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/r5/gemm_dp${dp}_tests.log 2>&1 || { echo "tests failed dp=$dp"; tail -20 gpurun_out/r5/gemm_dp${dp}_tests.log; exit 1; }
done
for dp in 0 1 2 3; do
  KUBEML_GEMM8_DP=$dp timeout -k 10 200 python -u tools/gemm_bench.py --tokens 16384 --rounds 5 --tiles 256x256x8,256x192x8 --shapes "$SH" > gpurun_out/r5/gemm_dp${dp}.jsonl 2>/dev/null || exit 1
done
python - <<'PY'
import json
for dp in range(4):
    print("DP", dp)
    for l in open(f'gpurun_out/r5/gemm_dp{dp}.jsonl'):
        d=json.loads(l)
        if d.get('summary'): print(' ', d); continue
        a=d['all_us']; print('  ', d['layout'], d['M'], d['N'], d['K'], 'torch', d['torch_us'], {k:v for k,v in a.items() if k!='torch'})
PY
