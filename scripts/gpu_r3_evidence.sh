#!/bin/bash
# Round-3 evidence at HEAD: ResNet-34 kernel trace, convergence parity, comm probe -> plan,
# 1-rank comm rehearsals, secondary configs (ResNet-50 K-AVG, BERT-base, VGG-16 elastic path).
set -o pipefail
out=gpurun_out/r3ev
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() { echo "== $1 $(date +%T)"; }

step trace
rm -rf $out/r34
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/r34 -o run -- python bench.py --steps 20 --warmup 3 --no-epoch --e2e off > $out/r34.log 2>&1 || { tail -20 $out/r34.log; exit 1; }
db=$(find $out/r34 -name "*.db" | head -1)
python tools/rocpd_summary.py $db --steps 24 --top 50 > $out/r34_summary.md && python tools/rocpd_timeline.py $db --first-kernel k_augment --nth -2 > $out/r34_timeline.md
rm -rf $out/r34
tail -1 $out/r34_timeline.md

step convergence
timeout -k 10 500 python -u tools/convergence_check.py --steps 1200 --out $out/convergence.json > $out/convergence.log 2>&1 || { tail -20 $out/convergence.log; exit 1; }
tail -2 $out/convergence.log | cut -c1-400

step probe
timeout -k 10 600 python -u tools/interference_probe.py --wires fp32,bf16 --out $out/interference.json --plan-out $out/comm_plan.json > $out/probe.log 2>&1 || { tail -20 $out/probe.log; exit 1; }
tail -3 $out/probe.log | cut -c1-600

step rehearsals
for plan in peer:end:fp32:256 rccl:overlap:fp32 rccl:end:fp32; do
  timeout -k 10 150 python bench.py --steps 100 --warmup 10 --force-comm --comm-plan $plan --no-epoch --e2e off > $out/fc_$plan.json 2> $out/fc.err || { tail -20 $out/fc.err; exit 1; }
  echo "$plan $(python -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['ms_per_step'])" $out/fc_$plan.json)"
done

step r50
timeout -k 10 300 python -u tools/bench_resnet50.py --force-comm > $out/r50.json 2> $out/r50.err || { tail -20 $out/r50.err; exit 1; }
tail -1 $out/r50.json | cut -c1-400
step bert
timeout -k 10 300 python -u tools/bench_bert.py > $out/bert.json 2> $out/bert.err || { tail -20 $out/bert.err; exit 1; }
tail -1 $out/bert.json | cut -c1-400
step vgg
timeout -k 10 400 python -u tools/run_elastic.py --gpus 1 --function vgg16 --policy scripted:1 --epochs 2 > $out/vgg.json 2> $out/vgg.err || { tail -20 $out/vgg.err; exit 1; }
tail -3 $out/vgg.json | cut -c1-600
echo done
