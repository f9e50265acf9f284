#!/bin/bash
# round 6: BN apply / backward-apply bandwidth and PMC at ResNet-50 shapes (tools/bn_bw.py)
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r6/bn${1:-}
mkdir -p $out
cd /tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/bn_bw.py > $out/bw.log 2>&1 || { tail -20 $out/bw.log; exit 1; }
grep '"M"' $out/bw.log
rm -rf $out/p1 $out/p2
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $out/p1 -o run --output-format csv -- python tools/bn_bw.py > $out/p1.log 2>&1 || { tail -5 $out/p1.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $out/p2 -o run --output-format csv -- python tools/bn_bw.py > $out/p2.log 2>&1 || { tail -5 $out/p2.log; exit 1; }
python tools/pmc_table.py --match k_bn --top 12 $(find $out/p1 $out/p2 -name "*counter_collection.csv") > $out/pmc.md
cat $out/pmc.md
