set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_models_gpu.py -k "vgg" > gpurun_out/r4/vgg_test.log 2>&1 || { tail -40 gpurun_out/r4/vgg_test.log; exit 1; }
tail -3 gpurun_out/r4/vgg_test.log
timeout -k 10 200 python -u tools/bench_vgg.py > gpurun_out/r4/vgg_bench_fused.json 2> gpurun_out/r4/vgg_bench_fused.err || { tail -20 gpurun_out/r4/vgg_bench_fused.err; exit 1; }
cat gpurun_out/r4/vgg_bench_fused.json
cp kubeml_amd/ops/conv_tuning.json gpurun_out/r4/conv_tuning_before.json
timeout -k 10 800 python -u tools/tune_conv.py --model vgg16 --batch 128 --reps 10 --max-seconds 600 > gpurun_out/r4/tune_vgg.log 2>&1 || { tail -20 gpurun_out/r4/tune_vgg.log; exit 1; }
tail -2 gpurun_out/r4/tune_vgg.log
cp kubeml_amd/ops/conv_tuning.json gpurun_out/r4/conv_tuning_vgg.json
timeout -k 10 200 python -u tools/bench_vgg.py > gpurun_out/r4/vgg_bench_tuned.json 2> gpurun_out/r4/vgg_bench_tuned.err || { tail -20 gpurun_out/r4/vgg_bench_tuned.err; exit 1; }
cat gpurun_out/r4/vgg_bench_tuned.json
rm -rf gpurun_out/r4/e2e_trace
timeout -k 10 400 python -u tools/bench_e2e.py --epochs 4 --validate --trace gpurun_out/r4/e2e_trace > gpurun_out/r4/e2e_bench.log 2>&1 || { tail -30 gpurun_out/r4/e2e_bench.log; exit 1; }
tail -1 gpurun_out/r4/e2e_bench.log
python tools/trace_spans.py gpurun_out/r4/e2e_trace --top 20 > gpurun_out/r4/e2e_spans.txt && head -40 gpurun_out/r4/e2e_spans.txt
