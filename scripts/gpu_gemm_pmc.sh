#!/bin/bash
# PMC counter passes over the GEMM kernel (one counter group per run).
set -o pipefail
out=gpurun_out/gemm_pmc
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cfg in "256,256" "128,128,2"; do
  tag=$(echo $cfg | tr ',' 'x')
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA -d $out/p1_$tag -o run --output-format csv -- python tools/gemm_one.py --tile $cfg > $out/p1_$tag.log 2>&1 || { tail -5 $out/p1_$tag.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d $out/p2_$tag -o run --output-format csv -- python tools/gemm_one.py --tile $cfg > $out/p2_$tag.log 2>&1 || { tail -5 $out/p2_$tag.log; exit 1; }
done
find $out -name "*counter_collection.csv" | head
