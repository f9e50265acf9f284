set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 420 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_multirank_gpu.py tests/test_peer_gpu.py > gpurun_out/r4/multirank.log 2>&1 || { tail -60 gpurun_out/r4/multirank.log; exit 1; }
tail -15 gpurun_out/r4/multirank.log
timeout -k 10 240 python -u bench.py --steps 40 --warmup 5 --force-comm --no-epoch --e2e off --comm-plan peer:shard:fp32:256 > gpurun_out/r4/bench_shard1.json 2> gpurun_out/r4/bench_shard1.err || { tail -30 gpurun_out/r4/bench_shard1.err; exit 1; }
cat gpurun_out/r4/bench_shard1.json
timeout -k 10 240 python -u bench.py --steps 40 --warmup 5 --no-epoch --e2e off > gpurun_out/r4/bench_base.json 2> gpurun_out/r4/bench_base.err || { tail -30 gpurun_out/r4/bench_base.err; exit 1; }
cat gpurun_out/r4/bench_base.json
