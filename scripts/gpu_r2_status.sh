#!/bin/bash
# Round-2 status pass: GPU tests, 1-GPU bench, ResNet-34 and BERT kernel profiles, ResNet-50 bench.
set -o pipefail
out=gpurun_out
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?; tail -4 $out/gpu_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
cat $out/bench.json
bash scripts/gpu_prof_r34.sh || exit 1
bash scripts/gpu_bert_prof3.sh || exit 1
timeout -k 10 300 python tools/bench_resnet50.py > $out/r50.log 2>&1 || { tail -5 $out/r50.log; exit 1; }
tail -3 $out/r50.log
