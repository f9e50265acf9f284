#!/bin/bash
# round 6: BN padded coefficient slots + two-level row fold vs HEAD (_abbase): tests, kernel
# bandwidth, LDS conflicts, ResNet-50 and ResNet-34 steps (alternating)
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r6/bnab
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for t in new base; do
  root=$GRAFT_REPO_ROOT; [ $t = base ] && root=$GRAFT_REPO_ROOT/_abbase
  (cd $root && timeout -k 10 200 python -u tools/bn_bw.py > $out/bw_$t.log 2>&1) || { tail -20 $out/bw_$t.log; exit 1; }
  echo "== $t"; grep '"M"' $out/bw_$t.log | cut -c1-150
done
rm -rf $out/p1
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $out/p1 -o run --output-format csv -- python tools/bn_bw.py > $out/p1.log 2>&1 || { tail -5 $out/p1.log; exit 1; }
python tools/pmc_table.py --match k_bn --top 12 $(find $out/p1 -name "*counter_collection.csv") > $out/pmc_new.md
cat $out/pmc_new.md
for rep in 1 2; do
  for t in new base; do
    root=$GRAFT_REPO_ROOT; [ $t = base ] && root=$GRAFT_REPO_ROOT/_abbase
    (cd $root && timeout -k 10 300 python -u tools/bench_resnet50.py > $out/r50_${t}_$rep.log 2>&1) || { tail -20 $out/r50_${t}_$rep.log; exit 1; }
    echo "r50 $t $rep $(tail -1 $out/r50_${t}_$rep.log | cut -c1-160)"
    (cd $root && timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-epoch --e2e off > $out/r34_${t}_$rep.json 2>/dev/null) || exit 1
    echo "r34 $t $rep $(tail -1 $out/r34_${t}_$rep.json | python -c "import json,sys;print(json.loads(sys.stdin.read())['ms_per_step'])")"
  done
done
