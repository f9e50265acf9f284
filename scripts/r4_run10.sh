set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 200 python -u bench.py --steps 60 --warmup 5 --no-epoch --e2e off > gpurun_out/r4/b_base.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/r4/b_base.json'));print('base', d['ms_per_step'])"
for b in 512 1024 2048; do
timeout -k 10 200 python -u bench.py --steps 60 --warmup 5 --force-comm --no-epoch --e2e off --comm-plan peer:shard:fp32:$b > gpurun_out/r4/b_shard_$b.json 2> gpurun_out/r4/b_shard_$b.err || { tail -30 gpurun_out/r4/b_shard_$b.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r4/b_shard_$b.json'));print($b, d['ms_per_step'], d.get('allreduce_ms'))"
done
timeout -k 10 200 python -u bench.py --steps 60 --warmup 5 --force-comm --no-epoch --e2e off --comm-plan peer:shard:fp32:2048 --comm-timing 0 > gpurun_out/r4/b_shard_nostamp.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/r4/b_shard_nostamp.json'));print('nostamp', d['ms_per_step'])"
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_multirank_gpu.py > gpurun_out/r4/multirank.log 2>&1 || { tail -40 gpurun_out/r4/multirank.log; exit 1; }
tail -1 gpurun_out/r4/multirank.log
