#!/bin/bash
set -o pipefail
out=gpurun_out/attnpmc3
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python tools/attn_micro.py --reps 5"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS -d $out/p1 -o run --output-format csv -- $B > $out/p1.log 2>&1 || { tail -5 $out/p1.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $out/p2 -o run --output-format csv -- $B > $out/p2.log 2>&1 || { tail -5 $out/p2.log; exit 1; }
python tools/pmc_summary.py $(find $out/p1 $out/p2 -name "*counter_collection.csv") --match attn > $out/attn.md
cat $out/attn.md
rm -rf $out/p1 $out/p2
