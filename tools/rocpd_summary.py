"""Summarise a rocprofv3 rocpd SQLite database (``--kernel-trace`` output) as markdown.

Usage: python tools/rocpd_summary.py <run_results.db> [--steps N] [--top 40] > profiles/x.md

Groups dispatches by demangled kernel name (template args kept, parameter list cut),
reports calls, total/avg time and share of GPU kernel time; with --steps, also per-step
time (total / N) — pass the number of profiled steps incl. warmup for a per-step view.
"""
import argparse
import re
import sqlite3


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    depth, out = 0, []
    # cut the parameter list: first '(' at template depth 0 after the name start
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0 and i > 0:
            break
        out.append(ch)
    s = "".join(out).replace("void ", "")
    return s if len(s) < 110 else s[:107] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=0)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, duration from kernels").fetchall()
    agg = {}
    for n, d in rows:
        k = short(n)
        e = agg.setdefault(k, [0, 0.0])
        e[0] += 1
        e[1] += d / 1e3  # ns -> us
    tot = sum(v[1] for v in agg.values())
    print(f"Total kernel time: {tot / 1e3:.3f} ms over {len(rows)} dispatches")
    if a.steps:
        print(f"Per step (÷{a.steps}): {tot / 1e3 / a.steps:.3f} ms")
    print()
    print("| kernel | calls | total us | avg us | % |")
    print("|---|---:|---:|---:|---:|")
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"| `{k}` | {n} | {t:.1f} | {t / n:.2f} | {100 * t / tot:.1f} |")


if __name__ == "__main__":
    main()
