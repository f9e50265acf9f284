#!/bin/bash
set -o pipefail
out=gpurun_out/g8b
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $out/gemm_tests.log 2>&1
rc=$?; tail -3 $out/gemm_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/gemm_bench.py --rounds 5 --reps 5 --tiles 256x256x8,256x256x4,128x128x2 \
  --shapes "0:8192:8192:8192;2:3072:768:16384;0:16384:3072:768;1:16384:768:3072;0:16384:768:3072;0:16384:3072:64" > $out/bench.log 2>&1 || { tail -5 $out/bench.log; exit 1; }
grep '^{' $out/bench.log | python -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l)
    if r.get('summary'): continue
    print(r['layout'], r['M'], r['N'], r['K'], 'torch', r['torch_us'], r['torch_TF'], r['all_us'])
"
args="--layout 0 --M 8192 --N 8192 --K 8192 --tile 256,256,8"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA -d $out/p1 -o run --output-format csv -- python tools/gemm_one.py $args --reps 5 > $out/p1.log 2>&1 || { tail -5 $out/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d $out/p2 -o run --output-format csv -- python tools/gemm_one.py $args --reps 5 > $out/p2.log 2>&1 || { tail -5 $out/p2.log; exit 1; }
python tools/pmc_summary.py $(find $out/p1 $out/p2 -name "*counter_collection.csv") --match k_gemm8
