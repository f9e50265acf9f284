#!/bin/bash
set -o pipefail
out=gpurun_out/r34lds
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python bench.py --steps 5 --warmup 2 --no-epoch"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $out/p1 -o run --output-format csv -- $B > $out/p1.log 2>&1 || { tail -5 $out/p1.log; exit 1; }
python tools/pmc_summary.py $(find $out/p1 -name "*counter_collection.csv") --match conv > $out/lds.md
cat $out/lds.md
rm -rf $out/p1
