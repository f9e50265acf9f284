#!/bin/bash
# Round-2 evidence: kernel-trace summaries + per-step timelines of the three workloads and a
# PMC counter table for the headline step (each counter group in its own run).
set -o pipefail
out=gpurun_out/prof_r2
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run_trace() {  # name first_kernel cmd...
  local name=$1 first=$2; shift 2
  rm -rf $out/$name
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name -o run -- "$@" > $out/$name.log 2>&1 || { tail -20 $out/$name.log; return 1; }
  local db=$(find $out/$name -name "*.db" | head -1)
  python tools/rocpd_summary.py $db --steps ${STEPS:-1} --top 40 > $out/${name}_summary.md || return 1
  python tools/rocpd_timeline.py $db --first-kernel $first --nth -2 > $out/${name}_timeline.md || return 1
  rm -rf $out/$name
  tail -1 $out/${name}_timeline.md
}
STEPS=24 run_trace r34 k_augment python bench.py --steps 20 --warmup 3 --no-epoch || exit 1
STEPS=5 run_trace bert k_embed_fwd python tools/bench_bert.py --steps 3 --warmup 1 || exit 1
STEPS=10 run_trace r50 k_augment python tools/bench_resnet50.py --steps 8 --warmup 2 --K 8 || exit 1
B="python bench.py --steps 5 --warmup 2 --no-epoch"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA -d $out/p1 -o run --output-format csv -- $B > $out/p1.log 2>&1 || { tail -5 $out/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE FETCH_SIZE -d $out/p2 -o run --output-format csv -- $B > $out/p2.log 2>&1 || { tail -5 $out/p2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $out/p3 -o run --output-format csv -- $B > $out/p3.log 2>&1 || { tail -5 $out/p3.log; exit 1; }
python tools/pmc_table.py --steps 7 --top 14 $(find $out/p1 $out/p2 $out/p3 -name "*counter_collection.csv") > $out/r34_pmc.md || exit 1
rm -rf $out/p1 $out/p2 $out/p3
cat $out/r34_pmc.md
