"""Print the kernel timeline of one training step from a rocprofv3 rocpd database:
name, grid, workgroup, VGPRs, duration and the idle gap before each dispatch.

Usage: python tools/rocpd_timeline.py <run_results.db> --first-kernel k_augment [--nth -2]
(the step is cut at consecutive dispatches of --first-kernel; --nth picks which step)."""
import argparse
import sqlite3

from rocpd_summary import short


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--first-kernel", default="k_augment")
    ap.add_argument("--nth", type=int, default=-2)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, grid_x, workgroup_x, vgpr_count, accum_vgpr_count, lds_size "
                     "from kernels order by start").fetchall()
    starts = [i for i, r in enumerate(rows) if a.first_kernel in r[0]]
    s0, s1 = starts[a.nth], (starts[a.nth + 1] if a.nth + 1 < 0 or a.nth + 1 < len(starts) else len(rows))
    step = rows[s0:s1]
    t0 = step[0][1]
    busy = gaps = 0.0
    prev_end = None
    print("| # | kernel | blocks | wg | vgpr | lds | us | gap us |")
    print("|---:|---|---:|---:|---:|---:|---:|---:|")
    for i, (n, st, en, gx, wx, vg, ag, lds) in enumerate(step):
        gap = (st - prev_end) / 1e3 if prev_end is not None else 0.0
        d = (en - st) / 1e3
        busy += d
        gaps += max(gap, 0.0)
        prev_end = en
        print(f"| {i} | `{short(n)[:70]}` | {gx // max(wx, 1)} | {wx} | {vg}+{ag} | {lds} | {d:.2f} | {gap:.2f} |")
    print(f"\nstep span {(step[-1][2] - t0) / 1e3:.1f} us, kernel busy {busy:.1f} us, gaps {gaps:.1f} us, "
          f"{len(step)} dispatches")


if __name__ == "__main__":
    main()
