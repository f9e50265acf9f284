#!/bin/bash
# round 6: every packed-rank case's numbers (no stop at the first failure), twice
set -o pipefail
export TMPDIR=/tmp
export KUBEML_PEER_TIMEOUT_S=20
out=$GRAFT_REPO_ROOT/gpurun_out/r6/shardride
mkdir -p $out
for rep in 1 2; do
  timeout -k 10 300 python -u tools/diag/mr_probe.py --world 2 > $out/mr_probe_$rep.log 2>&1 || { tail -40 $out/mr_probe_$rep.log; exit 1; }
  grep " rel " $out/mr_probe_$rep.log
done
