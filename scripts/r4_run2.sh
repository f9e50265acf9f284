set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
for b in 512 1024 2048; do
timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --force-comm --no-epoch --e2e off --comm-plan peer:shard:fp32:$b > gpurun_out/r4/bench_shard_$b.json 2> gpurun_out/r4/bench_shard_$b.err || { tail -30 gpurun_out/r4/bench_shard_$b.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r4/bench_shard_$b.json'));print($b, d['ms_per_step'], d.get('allreduce_ms'))"
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_e2e_gpu.py -k "share_one_gpu or elastic_one_two" > gpurun_out/r4/e2e_packed.log 2>&1 || { tail -80 gpurun_out/r4/e2e_packed.log; exit 1; }
tail -8 gpurun_out/r4/e2e_packed.log
timeout -k 10 900 python -u tools/convergence_multirank.py --out gpurun_out/r4/convergence_multirank.json > gpurun_out/r4/conv.log 2>&1 || { tail -40 gpurun_out/r4/conv.log; exit 1; }
tail -3 gpurun_out/r4/conv.log
