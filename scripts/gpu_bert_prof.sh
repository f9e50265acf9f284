set -o pipefail
out=gpurun_out
mkdir -p $out
timeout -k 10 200 python bench.py > $out/b_default.json 2> $out/b.err || exit 1
cat $out/b_default.json
timeout -k 10 200 python bench.py --steps 100 --force-comm --graph-comm on > $out/b_gc.json 2>> $out/b.err || exit 1
tail -1 $out/b_gc.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_bert -o run -- python tools/bench_bert.py --batch 32 --steps 5 --warmup 2 > $out/prof_bert.log 2>&1 || exit 1
echo done
