#!/bin/bash
# library-GEMM routing shipped in gemm_tuning.json: GEMM / BERT / transformer tests, the fused
# K-AVG and GELU kernels, BERT bench x2, then the ResNet-50 K-AVG rehearsals
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_bert_gpu.py tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread > $out/r33_tests.log 2>&1 || { tail -30 $out/r33_tests.log; exit 1; }
tail -1 $out/r33_tests.log
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "kavg or gelu" > $out/r33_kavg.log 2>&1 || { tail -30 $out/r33_kavg.log; exit 1; }
tail -1 $out/r33_kavg.log
for i in 1 2; do
  timeout -k 10 300 python -u tools/bench_bert.py > $out/bert_r33_$i.json 2> $out/bert_r33.err || { tail -20 $out/bert_r33.err; exit 1; }
  python -c "import json;d=json.load(open('$out/bert_r33_$i.json'));print('bert', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/pbert33 -o run -- python tools/bench_bert.py --steps 3 --warmup 1 > $out/pbert33.log 2>&1 || { tail -20 $out/pbert33.log; exit 1; }
bash scripts/r4_run30.sh
