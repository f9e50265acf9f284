#!/bin/bash
# round 6: BN coefficient-slot padding (stride 4 mod 32) vs HEAD (_abbase): tests, bandwidth, conflicts
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r6/bnab2
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for t in new base; do
  root=$GRAFT_REPO_ROOT; [ $t = base ] && root=$GRAFT_REPO_ROOT/_abbase
  (cd $root && timeout -k 10 200 python -u tools/bn_bw.py > $out/bw_$t.log 2>&1) || { tail -20 $out/bw_$t.log; exit 1; }
  echo "== $t"; grep '"M"' $out/bw_$t.log | cut -c1-150
  rm -rf $out/p_$t
  (cd $root && timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $out/p_$t -o run --output-format csv -- python tools/bn_bw.py > $out/p_$t.log 2>&1) || { tail -5 $out/p_$t.log; exit 1; }
  python tools/pmc_table.py --match k_bn --top 12 $(find $out/p_$t -name "*counter_collection.csv") > $out/pmc_$t.md
  cat $out/pmc_$t.md
done
