#!/bin/bash
# Round-3 closing evidence at HEAD.
set -o pipefail
out=gpurun_out/final3
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() { echo "== $1 $(date +%T)"; }
step smoke
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -5 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $out/gputests.log 2>&1
rc=$?; tail -2 $out/gputests.log; [ $rc = 0 ] || exit $rc
step bench
timeout -k 10 300 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print(d['ms_per_step'], d['value'], d['epoch_time_s'], d.get('e2e_epoch_time_s'), d.get('e2e_vs_bench_step_rate'))"
step rehearsal
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --force-comm --no-epoch --e2e off > $out/fc_auto.json 2> $out/fc.err || { tail -5 $out/fc.err; exit 1; }
python -c "import json;d=json.load(open('$out/fc_auto.json'));print(d['ms_per_step'], d['config'].get('comm_plan'), d['config'].get('comm_plan_source'))"
step trace
bash scripts/gpu_trace_now.sh || exit 1
step pmc
bash scripts/gpu_r34_pmc3.sh > $out/pmc.log 2>&1 || { tail -5 $out/pmc.log; exit 1; }
head -8 gpurun_out/r34pmc3/pmc_table.md
step convergence
timeout -k 10 600 python -u tools/convergence_check.py --steps 2000 --out $out/convergence.json > $out/convergence.log 2>&1 || { tail -20 $out/convergence.log; exit 1; }
tail -1 $out/convergence.log | cut -c1-300
step secondary
timeout -k 10 300 python -u tools/bench_bert.py > $out/bert.json 2> $out/bert.err || { tail -5 $out/bert.err; exit 1; }
tail -1 $out/bert.json | cut -c1-200
timeout -k 10 300 python -u tools/bench_resnet50.py --force-comm > $out/r50.json 2> $out/r50.err || { tail -5 $out/r50.err; exit 1; }
tail -1 $out/r50.json | cut -c1-200
echo done
