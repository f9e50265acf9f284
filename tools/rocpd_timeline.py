"""Print the kernel timeline of one training step from a rocprofv3 rocpd database:
name, FULL grid (x*y*z workgroups), workgroup size, a CU-fill column, VGPRs, LDS, duration and
the idle gap before each dispatch.

CU fill = min(workgroups, 256) / 256: the share of the 256 CUs that receive any work (< 1.0: part
of the chip idles for the whole dispatch).  Waves = workgroups / (256 CUs x resident workgroups per
CU), the per-CU residency bounded by LDS (160 KiB per CU), VGPRs (512 per SIMD lane budget, 4 SIMDs)
and 8 workgroups of <= 256 threads: < 1.0 means every workgroup is resident at once (the CUs run
below their occupancy limit), > 1.0 that the grid runs in several waves.

Usage: python tools/rocpd_timeline.py <run_results.db> --first-kernel k_augment [--nth -2]
(the step is cut at consecutive dispatches of --first-kernel; --nth picks which step)."""
import argparse
import sqlite3

from rocpd_summary import short

CUS = 256
LDS_PER_CU = 160 * 1024


def resident_per_cu(wg_threads, vgpr, agpr, lds):
    """Workgroups one CU can hold at once for this kernel's resources (an estimate)."""
    waves = max(1, -(-wg_threads // 64))
    regs = max(8, (vgpr or 0) + (agpr or 0))
    regs = -(-regs // 8) * 8
    waves_per_simd = max(1, min(8, 512 // regs))
    by_vgpr = (4 * waves_per_simd) // waves
    by_lds = LDS_PER_CU // lds if lds else 8
    by_thr = max(1, 1024 // max(wg_threads, 1)) if wg_threads > 256 else 8
    return max(1, min(by_vgpr, by_lds, by_thr, 8))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--first-kernel", default="k_augment")
    ap.add_argument("--nth", type=int, default=-2)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = {r[1] for r in c.execute("pragma table_info(kernels)").fetchall()}
    gy = "grid_y" if "grid_y" in cols else "1"
    gz = "grid_z" if "grid_z" in cols else "1"
    wy = "workgroup_y" if "workgroup_y" in cols else "1"
    wz = "workgroup_z" if "workgroup_z" in cols else "1"
    rows = c.execute(f"select name, start, end, grid_x, {gy}, {gz}, workgroup_x, {wy}, {wz}, vgpr_count, "
                     "accum_vgpr_count, lds_size from kernels order by start").fetchall()
    starts = [i for i, r in enumerate(rows) if a.first_kernel in r[0]]
    s0, s1 = starts[a.nth], (starts[a.nth + 1] if a.nth + 1 < 0 or a.nth + 1 < len(starts) else len(rows))
    step = rows[s0:s1]
    t0 = step[0][1]
    busy = gaps = 0.0
    prev_end = None
    under = 0.0
    print("| # | kernel | workgroups (x*y*z) | wg threads | CU fill | waves | vgpr | lds | us | gap us |")
    print("|---:|---|---:|---:|---:|---:|---:|---:|---:|---:|")
    for i, (n, st, en, gx, gyv, gzv, wx, wyv, wzv, vg, ag, lds) in enumerate(step):
        gap = (st - prev_end) / 1e3 if prev_end is not None else 0.0
        d = (en - st) / 1e3
        busy += d
        gaps += max(gap, 0.0)
        prev_end = en
        # rocprofv3 reports the grid in work-items: workgroups = ceil(grid / workgroup) per dimension
        nx = -(-gx // max(wx, 1))
        ny = -(-(gyv or 1) // max(wyv or 1, 1))
        nz = -(-(gzv or 1) // max(wzv or 1, 1))
        wgs = nx * ny * nz
        thr = max(wx, 1) * max(wyv or 1, 1) * max(wzv or 1, 1)
        fill = min(wgs, CUS) / CUS
        waves = wgs / (CUS * resident_per_cu(thr, vg, ag, lds))
        if wgs < CUS:
            under += d
        grid = f"{wgs} ({nx}*{ny}*{nz})" if ny * nz > 1 else f"{wgs}"
        print(f"| {i} | `{short(n)[:70]}` | {grid} | {thr} | {fill:.2f} | {waves:.2f} | {vg}+{ag} | {lds} | {d:.2f} | {gap:.2f} |")
    print(f"\nstep span {(step[-1][2] - t0) / 1e3:.1f} us, kernel busy {busy:.1f} us, gaps {gaps:.1f} us, "
          f"{len(step)} dispatches; {under:.1f} us in dispatches of fewer workgroups than CUs")


if __name__ == "__main__":
    main()
