#!/bin/bash
# Diagnostics: convergence parity on the harder task, framework-path epoch with worker traces, ResNet-50 trace.
set -o pipefail
out=gpurun_out/r3diag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
echo "== e2e $(date +%T)"
timeout -k 10 400 python -u tools/bench_e2e.py --epochs 4 --validate --trace $out/e2e_trace > $out/e2e.json 2> $out/e2e.err || { tail -20 $out/e2e.err; exit 1; }
cut -c1-900 $out/e2e.json
echo "== r50 $(date +%T)"
rm -rf $out/p50
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/p50 -o run -- python tools/bench_resnet50.py --steps 8 --warmup 2 --K 8 > $out/p50.log 2>&1 || { tail -20 $out/p50.log; exit 1; }
db=$(find $out/p50 -name "*.db" | head -1)
python tools/rocpd_summary.py $db --steps 10 --top 40 > $out/r50_summary.md && python tools/rocpd_timeline.py $db --first-kernel k_augment --nth -2 > $out/r50_timeline.md
rm -rf $out/p50
head -30 $out/r50_summary.md
echo "== convergence $(date +%T)"
timeout -k 10 600 python -u tools/convergence_check.py --steps 2000 --out $out/convergence.json > $out/convergence.log 2>&1 || { tail -20 $out/convergence.log; exit 1; }
grep acc $out/convergence.log | tail -12 | cut -c1-300
