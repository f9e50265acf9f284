set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
KUBEML_LOG_LEVEL=INFO timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_e2e_gpu.py -k "share_one_gpu or elastic_one_two" > gpurun_out/r4/e2e_packed.log 2>&1
echo "e2e rc=$?"
tail -5 gpurun_out/r4/e2e_packed.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_loader_gpu.py tests/test_multirank_gpu.py > gpurun_out/r4/loader_multirank.log 2>&1 || { tail -40 gpurun_out/r4/loader_multirank.log; exit 1; }
tail -3 gpurun_out/r4/loader_multirank.log
for b in 256 512; do
timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --force-comm --no-epoch --e2e off --comm-plan peer:shard:fp32:$b > gpurun_out/r4/bench_shard_$b.json 2> gpurun_out/r4/bench_shard_$b.err || { tail -30 gpurun_out/r4/bench_shard_$b.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r4/bench_shard_$b.json'));print($b, d['ms_per_step'], d.get('allreduce_ms'))"
done
rm -rf gpurun_out/r4/e2e_trace
timeout -k 10 400 python -u tools/bench_e2e.py --epochs 4 --validate --trace gpurun_out/r4/e2e_trace > gpurun_out/r4/e2e_bench.log 2>&1 || { tail -30 gpurun_out/r4/e2e_bench.log; exit 1; }
tail -1 gpurun_out/r4/e2e_bench.log
python tools/trace_spans.py gpurun_out/r4/e2e_trace > gpurun_out/r4/e2e_spans.txt && head -60 gpurun_out/r4/e2e_spans.txt
