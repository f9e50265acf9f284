#!/bin/bash
# timing-only experiment: KC half-tiles fetched as full 128-byte lines (KUBEML_GEMM8_FULL=1, wrong
# numerics) vs the shipped 64-byte half-line DMA; BERT shapes only (every dim a multiple of 256)
set -o pipefail
mkdir -p gpurun_out/r5
SH="0:16384:2304:768;1:16384:768:2304;0:16384:768:768;1:16384:768:768;0:16384:3072:768;1:16384:768:3072;0:16384:768:3072;1:16384:3072:768"
for r in 1 2; do
for f in 0 1; do
  KUBEML_GEMM8_FULL=$f timeout -k 10 200 python -u tools/gemm_bench.py --tokens 16384 --rounds 5 --tiles 256x256x8 --shapes "$SH" > gpurun_out/r5/gemm_full${f}_r$r.jsonl 2>/dev/null || exit 1
done
done
python - <<'PY'
import json
for r in (1,2):
  for f in (0,1):
    rows=[json.loads(l) for l in open(f'gpurun_out/r5/gemm_full{f}_r{r}.jsonl') if l.startswith('{')]
    print("run", r, "FULL", f, [(x['layout'], x['N'], x['K'], x['all_us'].get('256x256x8st/s1'), x['torch_us']) for x in rows if not x.get('summary')])
PY
