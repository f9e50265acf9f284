#!/bin/bash
# round 6: hand GEMM tiles vs hipBLASLt on the shapes the table still routes to the library
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r6/gemm
mkdir -p $out
S="0:16384:2304:768;1:16384:768:2304;0:16384:768:768;1:16384:768:768;0:16384:3072:768;1:16384:768:3072;0:16384:768:3072;1:16384:3072:768;0:2432:768:768;0:2432:30528:768;1:2432:768:30528;1:2432:768:768"
timeout -k 10 600 python -u tools/gemm_bench.py --shapes "$S" --rounds 5 --reps 10 > $out/blas_shapes.jsonl 2> $out/blas_shapes.err || { tail -20 $out/blas_shapes.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r6/gemm/blas_shapes.jsonl"):
    d = json.loads(l)
    if d.get("summary"):
        print(d); continue
    print(d["layout"], d["M"], d["N"], d["K"], "torch", d["torch_us"], "best", d["best"], d["best_us"], "x", d["speedup_vs_torch"])
PY
