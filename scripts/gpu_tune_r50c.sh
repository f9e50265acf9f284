#!/bin/bash
# Re-tune ResNet-50's weight-gradient plans (slab split-K since round 3) and pairs; bench before/after.
set -o pipefail
out=gpurun_out/r50tune
mkdir -p $out
timeout -k 10 300 python -u tools/bench_resnet50.py --force-comm > $out/before.json 2> $out/before.err || { tail -5 $out/before.err; exit 1; }
tail -1 $out/before.json | cut -c1-160
python - <<'PY'
import json
p = "kubeml_amd/ops/conv_tuning.json"
t = json.load(open(p))
px = {128 * s * s for s in (112, 56, 28, 14, 7)}
keep = []
for e in t["entries"]:
    w = e.get("wgrad")
    if e["mode"] == "wgrad" and e["Kd"] in px:
        continue
    if e["mode"] == "pair" and w and w[2] in px:
        continue
    keep.append(e)
print("dropped", len(t["entries"]) - len(keep))
t["entries"] = keep
json.dump(t, open("gpurun_out/r50tune/conv_tuning.json", "w"), indent=1)
PY
timeout -k 10 900 python -u tools/tune_conv.py --model resnet50 --batch 128 --size 224 --reps 5 --pairs --out $out/conv_tuning.json > $out/tune_r50.log 2>&1 || { tail -5 $out/tune_r50.log; exit 1; }
tail -2 $out/tune_r50.log
cp $out/conv_tuning.json kubeml_amd/ops/conv_tuning.json
timeout -k 10 300 python -u tools/bench_resnet50.py --force-comm > $out/after.json 2> $out/after.err || { tail -5 $out/after.err; exit 1; }
tail -1 $out/after.json | cut -c1-160
