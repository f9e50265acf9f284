#!/bin/bash
# PMC evidence: 1x1 weight gradient at (P 401408, K 128, C 256) on the implicit-GEMM wgrad vs the slab split-K GEMM
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/r4/pmc_wgrad
mkdir -p $out
for r in conv slab; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA -d $out/p1_$r -o run --output-format csv -- python tools/wgrad_one.py --route $r > $out/p1.log 2>&1 || { tail -5 $out/p1.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $out/p2_$r -o run --output-format csv -- python tools/wgrad_one.py --route $r > $out/p2.log 2>&1 || { tail -5 $out/p2.log; exit 1; }
  echo "== $r"
  python tools/pmc_summary.py $(find $out/p1_$r $out/p2_$r -name "*counter_collection.csv") > $out/summary_$r.txt
  cat $out/summary_$r.txt
done
