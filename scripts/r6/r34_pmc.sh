#!/bin/bash
# round 6: PMC passes over the headline ResNet-34 step (bench.py, 20 timed + 3 warm-up replays)
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r6/r34pmc
mkdir -p $out
cd /tmp && cd $GRAFT_REPO_ROOT
run() {  # tag counters...
  local tag=$1; shift
  rm -rf $out/$tag
  timeout -s KILL 150 rocprofv3 --pmc "$@" -d $out/$tag -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-epoch --e2e off > $out/$tag.log 2>&1 || { tail -5 $out/$tag.log; return 1; }
  echo "pass $tag ok"
}
run p1 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE && \
run p2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE && \
run p3 FETCH_SIZE && \
run p4 WRITE_SIZE && \
python tools/pmc_table.py --steps 24 --top 30 $(find $out/p1 $out/p2 $out/p3 $out/p4 -name "*counter_collection.csv") > $out/pmc.md && head -40 $out/pmc.md
