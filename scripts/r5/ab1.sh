#!/bin/bash
# same-box A/B of the fold paths and the BN apply grid (ms/step, 100 steps)
set -o pipefail
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/r5
mkdir -p $out
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --steps 100 --warmup 5 --no-epoch --e2e off > $out/ab_$label.json 2> $out/ab_$label.err || { tail -5 $out/ab_$label.err; return 1; }
  python -c "import json;d=json.loads(open('$out/ab_$label.json').read().strip().splitlines()[-1]);print('$label', d['ms_per_step'])"
}
for rep in 1 2; do
run none$rep KUBEML_BNB_FOLD=0 KUBEML_CROSS_FOLD=0 KUBEML_BNIN_ONESHOT=0 || exit 1
run all$rep KUBEML_BNB_FOLD=1 KUBEML_CROSS_FOLD=1 KUBEML_BNIN_ONESHOT=1 || exit 1
run cross$rep KUBEML_BNB_FOLD=0 KUBEML_CROSS_FOLD=1 KUBEML_BNIN_ONESHOT=0 || exit 1
run oneshot$rep KUBEML_BNB_FOLD=0 KUBEML_CROSS_FOLD=0 KUBEML_BNIN_ONESHOT=1 || exit 1
run bnb$rep KUBEML_BNB_FOLD=1 KUBEML_CROSS_FOLD=0 KUBEML_BNIN_ONESHOT=0 || exit 1
done
for vf in 2 4 8; do run vf$vf KUBEML_BNB_FOLD=0 KUBEML_CROSS_FOLD=0 KUBEML_BNIN_ONESHOT=0 KUBEML_BN_VMIN_FWD=$vf || exit 1; done
for vb in 2 4; do run vb$vb KUBEML_BNB_FOLD=0 KUBEML_CROSS_FOLD=0 KUBEML_BNIN_ONESHOT=0 KUBEML_BN_VMIN_BWD=$vb || exit 1; done
