#!/bin/bash
# PMC counters of the ResNet-50 step after the round-5 GEMM routes (3 passes, one counter group each) + kernel trace.
set -o pipefail
out=gpurun_out/r5/r50pmc
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python tools/bench_resnet50.py --steps 8 --warmup 8"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $out/p1 -o run --output-format csv -- $B > $out/p1.log 2>&1 || { tail -5 $out/p1.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE FETCH_SIZE GRBM_GUI_ACTIVE -d $out/p2 -o run --output-format csv -- $B > $out/p2.log 2>&1 || { tail -5 $out/p2.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d $out/p3 -o run --output-format csv -- $B > $out/p3.log 2>&1 || { tail -5 $out/p3.log; exit 1; }
for p in p1 p2 p3; do ls $(find $out/$p -name "*counter_collection.csv") > /dev/null || exit 1; done
python tools/pmc_table.py --steps 16 --top 24 $(find $out/p1 $out/p2 $out/p3 -name "*counter_collection.csv") > $out/pmc_table.md
cat $out/pmc_table.md
rm -rf $out/p1 $out/p2 $out/p3
