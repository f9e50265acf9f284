"""Every packed-rank train-step case of tests/test_multirank_gpu.py with its numbers printed (no stop
at the first failing assertion): relative error of the first update vs the single-process
reference, bit-identical ranks, finiteness, and the shard riders carried per rank.

    python tools/diag/mr_probe.py [--world 2] [--cases shardride,shardov]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--cases", default="", help="comma list of substrings of the case specs to run")
    a = ap.parse_args()
    import test_multirank_gpu as T
    cases = [c for c in T.CASES if not a.cases or any(s in c[0] + "/" + c[1] for s in a.cases.split(","))]
    res = T._spawn(a.world, cases)
    for key in res[0]:
        rs = [res[r][key] for r in range(a.world)]
        same = all(r["digests"] == rs[0]["digests"] for r in rs)
        print(key, "rel", rs[0].get("rel"), "rel_final", rs[0].get("rel_final"), "same", same, "finite", all(r["finite"] for r in rs),
              "ride", [(r.get("ride_slices"), r.get("ride_taken")) for r in rs], flush=True)


if __name__ == "__main__":
    main()
