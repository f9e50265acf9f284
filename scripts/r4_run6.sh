set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_multirank_gpu.py > gpurun_out/r4/multirank.log 2>&1 || { tail -40 gpurun_out/r4/multirank.log; exit 1; }
tail -3 gpurun_out/r4/multirank.log
for b in 256 512; do
timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --force-comm --no-epoch --e2e off --comm-plan peer:shard:fp32:$b > gpurun_out/r4/bench_shard_$b.json 2> gpurun_out/r4/bench_shard_$b.err || { tail -30 gpurun_out/r4/bench_shard_$b.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r4/bench_shard_$b.json'));print($b, d['ms_per_step'], d.get('allreduce_ms'))"
done
rm -rf gpurun_out/r4/e2e_trace
timeout -k 10 400 python -u tools/bench_e2e.py --epochs 4 --validate --trace gpurun_out/r4/e2e_trace > gpurun_out/r4/e2e_bench.log 2>&1 || { tail -30 gpurun_out/r4/e2e_bench.log; exit 1; }
tail -1 gpurun_out/r4/e2e_bench.log
python tools/trace_spans.py gpurun_out/r4/e2e_trace > gpurun_out/r4/e2e_spans.txt && head -60 gpurun_out/r4/e2e_spans.txt
timeout -k 10 200 python -u tools/bench_vgg.py > gpurun_out/r4/vgg_bench.json 2> gpurun_out/r4/vgg_bench.err || { tail -20 gpurun_out/r4/vgg_bench.err; exit 1; }
cat gpurun_out/r4/vgg_bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/vgg_prof -o vgg -- python tools/bench_vgg.py --steps 20 --warmup 3 > gpurun_out/r4/vgg_prof.log 2>&1 || { tail -20 gpurun_out/r4/vgg_prof.log; exit 1; }
find gpurun_out/r4/vgg_prof -name "*kernel_stats.csv" | head -3
