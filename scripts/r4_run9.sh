set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 500 python -u tools/tune_conv.py --model vgg16 --batch 128 --reps 10 --pairs --max-seconds 400 > gpurun_out/r4/tune_vgg_pairs.log 2>&1 || { tail -20 gpurun_out/r4/tune_vgg_pairs.log; exit 1; }
tail -1 gpurun_out/r4/tune_vgg_pairs.log
cp kubeml_amd/ops/conv_tuning.json gpurun_out/r4/conv_tuning_vgg_pairs.json
timeout -k 10 200 python -u tools/bench_vgg.py > gpurun_out/r4/vgg_bench_pairs.json 2> gpurun_out/r4/vgg_bench_pairs.err || { tail -20 gpurun_out/r4/vgg_bench_pairs.err; exit 1; }
cat gpurun_out/r4/vgg_bench_pairs.json
timeout -k 10 400 python -u tools/run_elastic.py --gpus 1 --function vgg16 --policy scripted:1 --epochs 3 > gpurun_out/r4/vgg_kubeml.log 2>&1 || { tail -30 gpurun_out/r4/vgg_kubeml.log; exit 1; }
tail -1 gpurun_out/r4/vgg_kubeml.log
timeout -k 10 400 python -u tools/bench_e2e.py --epochs 4 --validate > gpurun_out/r4/e2e_bench2.log 2>&1 || { tail -30 gpurun_out/r4/e2e_bench2.log; exit 1; }
tail -1 gpurun_out/r4/e2e_bench2.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/r4/vgg_prof2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/vgg_prof2 -o vgg -- python tools/bench_vgg.py --steps 20 --warmup 3 > gpurun_out/r4/vgg_prof2.log 2>&1 || { tail -20 gpurun_out/r4/vgg_prof2.log; exit 1; }
echo done
