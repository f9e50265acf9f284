#!/bin/bash
# Unrolled 2x2-map convs: numerics, ResNet-34 bench, tuning of the new 1x1 shapes, bench
# again with the tuned table, stock-PyTorch baseline (eager and graphed).
set -o pipefail
out=gpurun_out/unroll
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k unrolled -x -q --timeout 120 --timeout-method thread > $out/t_unroll.log 2>&1
rc=$?; tail -3 $out/t_unroll.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py tests/test_engine_gpu.py -x -q --timeout 150 --timeout-method thread > $out/t_models.log 2>&1
rc=$?; tail -3 $out/t_models.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-epoch > $out/bench_pre.json 2> $out/bench_pre.err || { tail -5 $out/bench_pre.err; exit 1; }
cat $out/bench_pre.json
cp kubeml_amd/ops/conv_tuning.json $out/conv_tuning.json
timeout -k 10 400 python -u tools/tune_conv.py --model resnet34 --batch 256 --out $out/conv_tuning.json > $out/tune.log 2>&1 || { tail -5 $out/tune.log; exit 1; }
timeout -k 10 400 python -u tools/tune_conv.py --model resnet34 --batch 256 --pairs --out $out/conv_tuning.json > $out/tune_pairs.log 2>&1 || { tail -5 $out/tune_pairs.log; exit 1; }
tail -4 $out/tune.log $out/tune_pairs.log
cp $out/conv_tuning.json kubeml_amd/ops/conv_tuning.json
timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-epoch > $out/bench_post.json 2> $out/bench_post.err || { tail -5 $out/bench_post.err; exit 1; }
cat $out/bench_post.json
timeout -k 10 200 python tools/stock_baseline.py --steps 50 --warmup 10 > $out/stock_eager.json 2>&1 || { tail -5 $out/stock_eager.json; exit 1; }
tail -1 $out/stock_eager.json
timeout -k 10 200 python tools/stock_baseline.py --steps 50 --warmup 10 --graph > $out/stock_graph.json 2>&1 || { tail -5 $out/stock_graph.json; exit 1; }
tail -1 $out/stock_graph.json
