#!/bin/bash
# k_gemm8 prefetch depth A/B: D = 5 (8 slots) vs D = 7 (10 slots, KUBEML_GEMM8_DEEP=1)
set -o pipefail
mkdir -p gpurun_out/r5
KUBEML_GEMM8_DEEP=1 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/r5/gemm_deep_tests.log 2>&1 || { tail -30 gpurun_out/r5/gemm_deep_tests.log; exit 1; }
tail -2 gpurun_out/r5/gemm_deep_tests.log
SH="0:16384:2304:768;1:16384:768:2304;0:16384:768:768;1:16384:768:768;0:16384:3072:768;1:16384:768:3072;0:16384:768:3072;1:16384:3072:768"
for r in 1 2; do
for d in 0 1; do
  KUBEML_GEMM8_DEEP=$d timeout -k 10 200 python -u tools/gemm_bench.py --tokens 16384 --rounds 5 --tiles 256x256x8 --shapes "$SH" > gpurun_out/r5/gemm_deep${d}_r$r.jsonl 2>/dev/null || exit 1
done
done
python - <<'PY'
import json
for r in (1,2):
  for d in (0,1):
    rows=[json.loads(l) for l in open(f'gpurun_out/r5/gemm_deep{d}_r{r}.jsonl') if l.startswith('{')]
    print("run", r, "DEEP", d, [(x['layout'], x['N'], x['K'], x['all_us'].get('256x256x8st/s1'), x['torch_us']) for x in rows if not x.get('summary')])
PY
