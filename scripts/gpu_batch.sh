#!/bin/bash
# GPU validation + measurements of the current tree (run under gpurun from the repo root).
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
out=gpurun_out
mkdir -p $out
echo "[gpu_batch] tests"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?
tail -4 $out/gpu_tests.log
[ $rc = 0 ] || exit $rc
echo "[gpu_batch] bench"
timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $out/bench.json 2> $out/bench.err || exit 1
cat $out/bench.json
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --segments on > $out/bench_seg.json 2>> $out/bench.err || exit 1
cat $out/bench_seg.json
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --force-comm --graph-comm off > $out/bench_fc.json 2>> $out/bench.err || exit 1
cat $out/bench_fc.json
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --force-comm --graph-comm on > $out/bench_gc.json 2>> $out/bench.err || exit 1
cat $out/bench_gc.json
echo "[gpu_batch] profile"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python bench.py --steps 20 --warmup 3 > $out/prof.log 2>&1 || exit 1
echo "[gpu_batch] gemm micro"
(cd tools && timeout -k 10 300 python gemm_micro.py > ../$out/gemm_micro.log 2>&1) || exit 1
tail -20 $out/gemm_micro.log
echo "[gpu_batch] resnet50"
timeout -k 10 400 python tools/bench_resnet50.py --steps 16 --warmup 8 > $out/bench_r50.json 2> $out/bench_r50.err || { tail -5 $out/bench_r50.err; exit 1; }
cat $out/bench_r50.json
echo "[gpu_batch] bert"
timeout -k 10 400 python tools/bench_bert.py --batch 32 --steps 10 --warmup 3 > $out/bench_bert.json 2> $out/bench_bert.err || { tail -5 $out/bench_bert.err; exit 1; }
cat $out/bench_bert.json
echo "[gpu_batch] done"
