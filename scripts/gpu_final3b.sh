#!/bin/bash
# Round-3 closing check after the attention rework: smoke, the whole GPU suite, PMC of the
# attention kernels.
set -o pipefail
out=gpurun_out/final3b
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() { echo "== $1 $(date +%T)"; }
step smoke
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -5 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $out/gputests.log 2>&1
rc=$?; tail -2 $out/gputests.log; [ $rc = 0 ] || exit $rc
step pmc
bash scripts/gpu_attn_pmc3.sh
