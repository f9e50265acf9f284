set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
cp kubeml_amd/ops/conv_tuning.json gpurun_out/r4/conv_tuning_before.json
timeout -k 10 800 python -u tools/tune_conv.py --model vgg16 --batch 128 --reps 10 --max-seconds 700 > gpurun_out/r4/tune_vgg.log 2>&1 || { tail -20 gpurun_out/r4/tune_vgg.log; exit 1; }
tail -2 gpurun_out/r4/tune_vgg.log
cp kubeml_amd/ops/conv_tuning.json gpurun_out/r4/conv_tuning_vgg.json
timeout -k 10 200 python -u tools/bench_vgg.py > gpurun_out/r4/vgg_bench2.json 2> gpurun_out/r4/vgg_bench2.err || { tail -20 gpurun_out/r4/vgg_bench2.err; exit 1; }
cat gpurun_out/r4/vgg_bench2.json
