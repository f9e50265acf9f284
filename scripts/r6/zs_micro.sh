#!/bin/bash
# round 6: shard-rider slices alone vs ranged SGD; shardov packed ranks after the classifier-flag fix
set -o pipefail
export TMPDIR=/tmp
export KUBEML_PEER_TIMEOUT_S=20
out=$GRAFT_REPO_ROOT/gpurun_out/r6/zs
mkdir -p $out
timeout -k 10 200 python -u tools/diag/zs_rider_micro.py > $out/micro.log 2>&1 || { tail -30 $out/micro.log; exit 1; }
grep stage $out/micro.log
timeout -k 10 240 python -u tools/diag/mr_probe.py --world 2 --cases shardov > $out/shardov.log 2>&1 || { tail -30 $out/shardov.log; exit 1; }
grep " rel " $out/shardov.log
