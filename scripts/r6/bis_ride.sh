#!/bin/bash
# round 6: shardov packed-rank numbers at 429a6b7 (bisect tree) and here, then shard vs shardride rehearsal
set -o pipefail
export TMPDIR=/tmp
export KUBEML_PEER_TIMEOUT_S=20
out=$GRAFT_REPO_ROOT/gpurun_out/r6/shardride
mkdir -p $out
(cd _bisect && timeout -k 10 240 python -u tools/diag/mr_probe.py --world 2 --cases shardov > $out/bisect_shardov.log 2>&1) || { tail -30 $out/bisect_shardov.log; exit 1; }
grep " rel " $out/bisect_shardov.log
timeout -k 10 240 python -u tools/diag/mr_probe.py --world 2 --cases shardov,shardride > $out/main_shardov.log 2>&1 || { tail -30 $out/main_shardov.log; exit 1; }
grep " rel " $out/main_shardov.log
bash scripts/r6/shardride2.sh
