#!/bin/bash
# round 6: rider micro, packed-rank shard riders (2 and 4 ranks), 1-rank rehearsal shard vs shardride
set -o pipefail
export TMPDIR=/tmp
export KUBEML_PEER_TIMEOUT_S=20
out=$GRAFT_REPO_ROOT/gpurun_out/r6/zs
mkdir -p $out
timeout -k 10 200 python -u tools/diag/zs_rider_micro.py > $out/micro2.log 2>&1 || { tail -30 $out/micro2.log; exit 1; }
grep stage $out/micro2.log
timeout -k 10 240 python -u tools/diag/mr_probe.py --world 2 --cases shardride,shardov > $out/p2.log 2>&1 || { tail -30 $out/p2.log; exit 1; }
grep " rel " $out/p2.log
timeout -k 10 240 python -u tools/diag/mr_probe.py --world 4 --cases shardride > $out/p4.log 2>&1 || { tail -30 $out/p4.log; exit 1; }
grep " rel " $out/p4.log
bash scripts/r6/shardride2.sh
