#!/bin/bash
# k_gemm8 diagnosis (timing only, numerics deliberately broken): 1 DMA from the zero page, 2 no MFMA,
# 3 no fragment reads, 4 no DMA, 5 no in-phase barriers
set -o pipefail
mkdir -p gpurun_out/r5
SH="0:16384:2304:768;1:16384:768:2304;0:16384:768:3072;1:16384:3072:768"
for ex in 0 1 2 3 4 5; do
  KUBEML_GEMM8_EXP=$ex timeout -k 10 200 python -u tools/gemm_bench.py --tokens 16384 --rounds 3 --tiles 256x256x8 --shapes "$SH" > gpurun_out/r5/gemm_exp${ex}.jsonl 2>/dev/null || { echo "exp $ex failed"; exit 1; }
done
python - <<'PY'
import json
for ex in range(6):
    r=[json.loads(l) for l in open(f'gpurun_out/r5/gemm_exp{ex}.jsonl')]
    print("EXP", ex, [(d['layout'], d['N'], d['K'], d['all_us'].get('256x256x8st/s1')) for d in r if not d.get('summary')])
PY
