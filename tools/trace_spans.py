"""Host-side span summary of KUBEML_TRACE Chrome traces: per task (``task:<kind>`` spans, in
time order), the total of every span name nested in it — where a task's wall time goes
(e.g. the first train task of a job against a steady one).

    python tools/trace_spans.py <trace dir> [--top 12]
"""
import argparse
import collections
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    evs = []
    for f in sorted(glob.glob(os.path.join(a.path, "*.json"))):
        for e in json.load(open(f)).get("traceEvents", []):
            if e.get("ph") == "X" and e.get("cat") != "gpu":
                e["file"] = os.path.basename(f)
                evs.append(e)
    tasks = sorted((e for e in evs if e["name"].startswith("task:")), key=lambda e: e["ts"])
    for t in tasks:
        t0, t1 = t["ts"], t["ts"] + t["dur"]
        inner = [e for e in evs if e is not t and e["pid"] == t["pid"] and t0 <= e["ts"] and e["ts"] + e["dur"] <= t1]
        tot = collections.Counter()
        cnt = collections.Counter()
        for e in inner:
            tot[e["name"]] += e["dur"]
            cnt[e["name"]] += 1
        print(f"{t['name']} {t['file']} epoch={t['args'].get('epoch')} wall={t['dur'] / 1e3:.1f} ms")
        for name, us in tot.most_common(a.top):
            print(f"    {name:24s} {us / 1e3:9.1f} ms  x{cnt[name]}")


if __name__ == "__main__":
    main()
