#!/bin/bash
# round 6: shard riders after the host re-plan + self-test: packed ranks (2, 4), multirank tests,
# 1-rank rehearsal (shard vs shardride, alternating) and the plan probe's predictions
set -o pipefail
export TMPDIR=/tmp
export KUBEML_PEER_TIMEOUT_S=20
out=$GRAFT_REPO_ROOT/gpurun_out/r6/zs3
mkdir -p $out
timeout -k 10 240 python -u tools/diag/mr_probe.py --world 2 --cases shardride > $out/p2.log 2>&1 || { tail -30 $out/p2.log; exit 1; }
grep " rel " $out/p2.log
timeout -k 10 240 python -u tools/diag/mr_probe.py --world 4 --cases shardride > $out/p4.log 2>&1 || { tail -30 $out/p4.log; exit 1; }
grep " rel " $out/p4.log
timeout -k 10 600 python -u -m pytest tests/test_multirank_gpu.py -x -q --timeout 300 --timeout-method thread > $out/mr.log 2>&1 || { tail -30 $out/mr.log; exit 1; }
tail -1 $out/mr.log
for rep in 1 2; do
  for plan in "peer:shard:fp32:1024" "peer:shardride:fp32:1024"; do
    tag=$(echo $plan | tr ':' '_')
    timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-epoch --e2e off --force-comm --comm-plan $plan > $out/b_${tag}_$rep.json 2> $out/b_${tag}_$rep.err || { tail -20 $out/b_${tag}_$rep.err; exit 1; }
    echo "plan=$plan rep=$rep $(tail -1 $out/b_${tag}_$rep.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'])")"
  done
done
grep -i "rider\|warn" $out/b_peer_shardride_fp32_1024_1.err | head -5
python tools/shard_plan_probe.py --from-dir $out > $out/probe.json
cat $out/probe.json
