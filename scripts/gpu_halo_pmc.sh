#!/bin/bash
# PMC counters of the halo-patch conv vs the tuned implicit-GEMM plan (tools/halo_micro.py).
set -o pipefail
out=gpurun_out/halopmc
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python tools/halo_micro.py --batch 256"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $out/kt -o run -- $B > $out/kt.log 2>&1 || { tail -5 $out/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $out/p1 -o run --output-format csv -- $B > $out/p1.log 2>&1 || { tail -5 $out/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE FETCH_SIZE GRBM_GUI_ACTIVE -d $out/p2 -o run --output-format csv -- $B > $out/p2.log 2>&1 || { tail -5 $out/p2.log; exit 1; }
python tools/pmc_table.py --steps 1 --top 20 $(find $out/p1 $out/p2 -name "*counter_collection.csv") > $out/pmc_table.md
cat $out/pmc_table.md
db=$(find $out/kt -name "*.db" | head -1)
python tools/rocpd_summary.py $db --top 20 > $out/kt_summary.md
head -30 $out/kt_summary.md
rm -rf $out/p1 $out/p2 $out/kt
