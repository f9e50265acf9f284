#!/bin/bash
# Round-2 closing evidence: whole GPU suite, driver smoke, headline bench (+ RCCL rehearsal),
# BERT / ResNet-50 benches, kernel-trace summaries + timelines of the three workloads.
set -o pipefail
out=gpurun_out/final
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?; tail -3 $out/gpu_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -5 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 200 python bench.py > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 200 python bench.py --force-comm --steps 100 --no-epoch > $out/bench_fc.json 2> $out/bench_fc.err || { tail -5 $out/bench_fc.err; exit 1; }
echo "force-comm lines=$(wc -l < $out/bench_fc.json) $(cut -c1-120 $out/bench_fc.json)"
timeout -k 10 300 python tools/bench_bert.py --steps 20 > $out/bert.json 2> $out/bert.err || { tail -5 $out/bert.err; exit 1; }
tail -1 $out/bert.json | cut -c1-200
timeout -k 10 300 python tools/bench_resnet50.py > $out/r50.log 2>&1 || { tail -5 $out/r50.log; exit 1; }
tail -1 $out/r50.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run_trace() {  # name first_kernel steps cmd...
  local name=$1 first=$2 steps=$3; shift 3
  rm -rf $out/$name
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name -o run -- "$@" > $out/$name.log 2>&1 || { tail -20 $out/$name.log; return 1; }
  local db=$(find $out/$name -name "*.db" | head -1)
  python tools/rocpd_summary.py $db --steps $steps --top 40 > $out/${name}_summary.md || return 1
  python tools/rocpd_timeline.py $db --first-kernel $first --nth -2 > $out/${name}_timeline.md || return 1
  rm -rf $out/$name
  tail -1 $out/${name}_timeline.md
}
run_trace r34 k_augment 24 python bench.py --steps 20 --warmup 3 --no-epoch || exit 1
run_trace bert k_embed_fwd 5 python tools/bench_bert.py --steps 3 --warmup 1 || exit 1
run_trace r50 k_augment 10 python tools/bench_resnet50.py --steps 8 --warmup 2 --K 8 || exit 1
