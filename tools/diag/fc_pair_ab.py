"""In-step A/B of the classifier's grouped backward plan (the 512 -> 1000 Linear run as a 1x1
conv: dgrad [256 x 512, K = 1000] + wgrad [1000 x 512, K = 256] in one k_conv_pair launch):
writes one tuning file per candidate (the shipped table + a pair entry for that shape) and times
bench.py's headline step with each, alternating with the shipped table.

    python tools/diag/fc_pair_ab.py [--reps 2]"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CANDS = [([32, 32, 64, 2, 0], [32, 32, 64, 1, 0]), ([32, 32, 64, 4, 0], [32, 32, 64, 1, 0]),
         ([32, 64, 64, 1, 0], [32, 32, 64, 1, 0]), ([32, 64, 64, 2, 0], [32, 32, 64, 1, 0]),
         ([32, 32, 64, 2, 0], [64, 32, 64, 1, 0]), ([32, 32, 64, 1, 0], [64, 32, 64, 1, 0])]


def step_ms(tune_file):
    env = dict(os.environ)
    if tune_file:
        env["KUBEML_CONV_TUNING_FILE"] = tune_file
    out = subprocess.run([sys.executable, "bench.py", "--steps", "200", "--warmup", "20", "--no-epoch", "--e2e", "off"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    if out.returncode:
        raise SystemExit(out.stderr[-2000:])
    return json.loads(out.stdout.strip().splitlines()[-1])["ms_per_step"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "r6", "fcpair"))
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    base = json.load(open(os.path.join(ROOT, "kubeml_amd", "ops", "conv_tuning.json")))
    files = []
    for i, (d, w) in enumerate(CANDS):
        t = json.loads(json.dumps(base))
        t["entries"].append({"mode": "pair", "M": 256, "N": 512, "Kd": 1000, "wgrad": [1000, 512, 256], "cfg": d,
                             "wcfg": w})
        f = os.path.join(a.out, f"tune_{i}.json")
        json.dump(t, open(f, "w"))
        files.append(f)
    for rep in range(a.reps):
        for i, f in enumerate(files):
            b = step_ms(None)
            c = step_ms(f)
            print(json.dumps({"rep": rep, "cand": CANDS[i], "ms": c, "base_ms": b}), flush=True)


if __name__ == "__main__":
    main()
