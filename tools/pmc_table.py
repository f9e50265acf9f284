"""Per-kernel PMC table from several rocprofv3 --pmc passes (one counter group per pass).

Sums every counter over the dispatches of one kernel name (summed over the per-XCD / SE
instances of each dispatch), divides by --steps, and derives:
  mfma_util  = SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMDs x 256 CUs x per-XCD GRBM_GUI_ACTIVE)
               (share of the chip's matrix-pipe cycles the kernel kept busy)
  lds_confl  = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  fetch_MB   = 2 x FETCH_SIZE (KB) / 1024  (gfx950 FETCH_SIZE reports half the bytes of
               wide coalesced reads: MI355X_MICROARCH.md "HBM")
  write_MB   = WRITE_SIZE (KB) / 1024
  wait_any / wait_inst / active = shares of SQ_WAVE_CYCLES

Usage: python tools/pmc_table.py --steps S --top 8 <counter_collection.csv>...
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name):
    m = re.search(r"((?:k_|__amd_)\w+(?:<[^()]*>)?)", name)
    return (m.group(1) if m else name.split("(")[0])[:80]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--steps", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=8)
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    tot = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    for path in a.csv:
        with open(path) as f:
            for r in csv.DictReader(f):
                name = r.get("Kernel_Name", "")
                if a.match not in name:
                    continue
                tot[name][r["Counter_Name"]] += float(r["Counter_Value"])
                calls[name].add((path, r["Dispatch_Id"]))
    npass = max(1, len(a.csv))
    ncalls = {k: len(v) / npass for k, v in calls.items()}
    key = "SQ_WAVE_CYCLES"
    order = sorted(tot, key=lambda k: -tot[k].get(key, 0.0))
    print("| kernel | calls/step | MFMA us/call/SIMD | MFMA insts/call | lds_confl | fetch MB/step | write MB/step | "
          "wait_any | wait_inst | active |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k in order[:a.top]:
        c = tot[k]
        s = a.steps
        n = max(1.0, ncalls[k])
        # matrix-pipe busy time of one SIMD per call, at ~2.1 GHz (compare with the call's trace time)
        mf_us = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / 1024.0 / n / 2.1e3
        mf_n = c.get("SQ_INSTS_MFMA", 0.0) / n
        ldsc = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"] if c.get("SQ_LDS_IDX_ACTIVE") else 0.0
        fetch = 2.0 * c.get("FETCH_SIZE", 0.0) / 1024.0 / s
        wr = c.get("WRITE_SIZE", 0.0) / 1024.0 / s
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        sh = lambda n: (c.get(n, 0.0) / wc) if wc else float("nan")
        nm = short(k)
        print(f"| `{nm}` | {ncalls[k] / s:.0f} | {mf_us:.2f} | {mf_n:.0f} | {ldsc:.1%} | {fetch:.1f} | {wr:.1f} | "
              f"{sh('SQ_WAIT_ANY'):.0%} | {sh('SQ_WAIT_INST_ANY'):.0%} | {sh('SQ_ACTIVE_INST_ANY'):.0%} |")


if __name__ == "__main__":
    main()
