#!/bin/bash
# round 6: implicit-GEMM K-contiguous LDS rows padded +16 (conflict-free fragment reads) vs _abbase
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r6/padk
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_engine_gpu.py tests/test_determinism_gpu.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
cd /tmp && cd $GRAFT_REPO_ROOT
rm -rf $out/p_new
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $out/p_new -o run --output-format csv -- python tools/bench_resnet50.py --steps 4 --warmup 2 > $out/p_new.log 2>&1 || { tail -5 $out/p_new.log; exit 1; }
python tools/pmc_table.py --steps 6 --top 14 $(find $out/p_new -name "*counter_collection.csv") > $out/pmc_new.md
cat $out/pmc_new.md
for rep in 1 2 3; do
  for t in new base; do
    root=$GRAFT_REPO_ROOT; [ $t = base ] && root=$GRAFT_REPO_ROOT/_abbase
    (cd $root && timeout -k 10 300 python -u tools/bench_resnet50.py > $out/r50_${t}_$rep.log 2>&1) || { tail -20 $out/r50_${t}_$rep.log; exit 1; }
    echo "r50 $t $rep $(tail -1 $out/r50_${t}_$rep.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'])")"
    (cd $root && timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-epoch --e2e off > $out/r34_${t}_$rep.json 2>/dev/null) || exit 1
    echo "r34 $t $rep $(tail -1 $out/r34_${t}_$rep.json | python -c "import json,sys;print(json.loads(sys.stdin.read())['ms_per_step'])")"
  done
done
