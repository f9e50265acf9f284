"""Summarise rocprofv3 --pmc counter CSVs: per kernel name, the median over dispatches of
each counter (summed over the per-XCD/SE instances of one dispatch).

Usage: python tools/pmc_summary.py <run_counter_collection.csv> [--match k_gemm]"""
import argparse
import csv
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # kernel -> counter -> dispatch -> sum
    for path in a.csv:
        with open(path) as f:
            for r in csv.DictReader(f):
                name = r.get("Kernel_Name", "")
                if a.match not in name:
                    continue
                per[name][r["Counter_Name"]][(path, r["Dispatch_Id"])] += float(r["Counter_Value"])
    for k, cs in per.items():
        short = k.split("(")[0][:90]
        print(f"## {short}")
        for c, d in sorted(cs.items()):
            v = sorted(d.values())
            print(f"  {c:28s} median {statistics.median(v):14.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
