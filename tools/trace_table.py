"""Render the device compute/comm timeline of a KUBEML_TRACE Chrome trace as a markdown table.

    python tools/trace_table.py <trace dir or .json> [--last 2] [--anchor "fwd+bwd seg0"]

Takes the ``gpu``-category spans (tracks ``gpu:compute`` / ``gpu:comm``, written by
``kubeml_amd.utils.trace.gpu_span``), keeps the last ``--last`` steps (a step starts at each
span named ``--anchor``, default: the name of the first span on the compute track) and prints
start / duration in µs relative to the first kept span, plus per-step totals: compute busy,
comm spans, and how much of the comm time overlaps compute.
"""
import argparse
import glob
import json
import os


def load(path):
    files = sorted(glob.glob(os.path.join(path, "*.json"))) if os.path.isdir(path) else [path]
    evs, tracks = [], {}
    for f in files:
        d = json.load(open(f))
        for e in d.get("traceEvents", []):
            if e.get("ph") == "M" and e.get("name") == "thread_name":
                tracks[(e["pid"], e["tid"])] = e["args"]["name"]
            elif e.get("ph") == "X" and e.get("cat") == "gpu":
                evs.append(e)
    for e in evs:
        e["track"] = tracks.get((e["pid"], e["tid"]), str(e["tid"]))
    return sorted(evs, key=lambda e: e["ts"])


def overlap(a0, a1, spans):
    return sum(max(0.0, min(a1, b1) - max(a0, b0)) for b0, b1 in spans)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--last", type=int, default=2)
    ap.add_argument("--anchor", default=None)
    a = ap.parse_args()
    evs = load(a.path)
    comp = [e for e in evs if e["track"].endswith("compute")]
    if not comp:
        raise SystemExit("no gpu:compute spans in the trace")
    anchor = a.anchor or comp[0]["name"]
    starts = [e["ts"] for e in comp if e["name"] == anchor]
    t0 = starts[-a.last] if len(starts) >= a.last else starts[0]
    keep = [e for e in evs if e["ts"] >= t0]
    print(f"Last {min(a.last, len(starts))} steps (µs, relative; a step starts at `{anchor}`):\n")
    print("| track | span | start | dur |")
    print("|---|---|---:|---:|")
    for e in keep:
        print(f"| {e['track'].split(':')[-1]} | {e['name']} | {e['ts'] - t0:.1f} | {e['dur']:.1f} |")
    bounds = [s for s in starts if s >= t0] + [float("inf")]
    print("\n| step | compute busy µs | comm µs | comm overlapped with compute µs | step span µs |")
    print("|---:|---:|---:|---:|---:|")
    for i in range(len(bounds) - 1):
        lo, hi = bounds[i], bounds[i + 1]
        st = [e for e in keep if lo <= e["ts"] < hi]
        cs = [(e["ts"], e["ts"] + e["dur"]) for e in st if e["track"].endswith("compute")]
        ms = [(e["ts"], e["ts"] + e["dur"]) for e in st if e["track"].endswith("comm")]
        busy = sum(b - a_ for a_, b in cs)
        comm = sum(b - a_ for a_, b in ms)
        ov = sum(overlap(a_, b, cs) for a_, b in ms)
        end = max(b for _, b in cs + ms)
        print(f"| {i} | {busy:.1f} | {comm:.1f} | {ov:.1f} | {end - lo:.1f} |")


if __name__ == "__main__":
    main()
