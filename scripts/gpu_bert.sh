#!/bin/bash
# BERT path check: linear tests, BERT tests, BERT bench, then a kernel-trace profile.
set -o pipefail
out=gpurun_out
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_bert_gpu.py -m gpu -x -q -k "linear or bert" --timeout 150 --timeout-method thread > $out/t_bert.log 2>&1
rc=$?
tail -4 $out/t_bert.log
[ $rc = 0 ] || exit $rc
timeout -k 10 200 python tools/wgrad_split.py > $out/wgrad_split.log 2>&1 || exit 1
cat $out/wgrad_split.log
timeout -k 10 300 python tools/bench_bert.py --batch 32 --steps 10 --warmup 3 > $out/bench_bert.json 2> $out/bench_bert.err || { tail -5 $out/bench_bert.err; exit 1; }
cat $out/bench_bert.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_bert -o run -- python tools/bench_bert.py --batch 32 --steps 5 --warmup 2 > $out/prof_bert.log 2>&1 || exit 1
echo done
