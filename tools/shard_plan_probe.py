"""ZeRO-1 plans on ONE MI355X -> predicted N-rank steps -> kubeml_amd/parallel/comm_plan.json.

Measured (1-rank group, ``bench.py --force-comm``: the peer kernels run, the link does not):
  base      the step with no collective
  shard     peer:shard:fp32:1024  — reduce-scatter + fused SGD + all-gather after the backward
  shardov:b peer:shardov:fp32:b   — the same per backward stage on a side stream (grid cap b)

N-rank prediction (the link is not measurable on one GPU; documented model):
  link(N)       = (4 + 2) (N - 1) / N * n_params / B_link      (fp32 reduce-scatter reads + bf16 all-gather
                                                                 reads per rank, B_link = aggregate xGMI read
                                                                 bandwidth of one GPU: 7 links)
  shard(N)      = t(shard) + link(N)                            (nothing overlaps it)
  shardov(N, b) = t(shardov b) + f_first * link(N) + max(0, (1 - f_first) link(N) - window)
                  f_first = the first stage's share of the bytes (stem + layer1: it cannot hide);
                  window  = the measured side-stream collective span at world 1 (what the backward
                  after the first stage leaves to hide in)
  shardride(N)  = t(shardride) + f_rest * link(N) + sum over the four rider phases of
                  max(0, bytes_phase(N) / B_link - host_window_phase)
                  (engine/dp.py ``shardride``: each phase's link bytes are read by rider blocks of
                  its host launches, so they hide in those launches' span; host windows from the
                  round-6 shardride timeline, profiles/r6/shardride.md; f_rest = layer2 + layer1 +
                  stem, the part still exchanged after the backward)
The smaller prediction per N becomes ``choice`` (ties keep "shard": no second queue).

  python tools/shard_plan_probe.py [--link-gbs 750] [--from-dir gpurun_out/r5] [--write]
``--from-dir`` reads existing ``reh_*.json`` / ``b_peer_*.json`` bench lines instead of running.
"""
import argparse
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PLAN = os.path.join(ROOT, "kubeml_amd", "parallel", "comm_plan.json")
N_PARAMS = 21_814_696          # ResNet-34, 1000 classes (flat fp32 space)
FIRST_STAGE_FRAC = 0.0107      # stem + layer1 parameters / all (models/resnet.py stages())
RIDE_A, RIDE_B = 13_627_392, 6_822_400   # layer4 + fc, layer3 (models/resnet.py comm_ride_plan())
# host-launch spans the rider phases hide in (us; profiles/r6/shardride.md): RS-A on layer3's 13
# conv-backward launches, AG-A on 4 of layer2's, RS-B on the other 5, AG-B on layer1's 6
RIDE_WINDOWS_US = {"rs_a": 220.0, "ag_a": 80.0, "rs_b": 100.0, "ag_b": 120.0}


def _bench(args):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "100", "--warmup", "5", "--no-epoch",
           "--e2e", "off"] + args
    out = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True, check=True).stdout
    return json.loads(out.strip().splitlines()[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--link-gbs", type=float, default=750.0,
                    help="aggregate xGMI read bandwidth of one GPU (7 links x ~153 GB/s at ~70%% efficiency)")
    ap.add_argument("--from-dir", default=None)
    ap.add_argument("--blocks", default="64,256")
    ap.add_argument("--write", action="store_true", help="update comm_plan.json")
    a = ap.parse_args()
    meas = {}
    if a.from_dir:
        for f in glob.glob(os.path.join(a.from_dir, "reh_*.json")) + glob.glob(os.path.join(a.from_dir, "b_peer_*.json")):
            d = json.loads(open(f).read().strip().splitlines()[-1])
            key = d["config"].get("comm_plan") or "base"
            meas.setdefault(key, []).append((d["ms_per_step"], d.get("allreduce_ms")))
    else:
        meas["base"] = [(_bench([])["ms_per_step"], None)]
        d = _bench(["--force-comm", "--comm-plan", "peer:shard:fp32:1024"])
        meas[d["config"]["comm_plan"]] = [(d["ms_per_step"], d.get("allreduce_ms"))]
        for b in a.blocks.split(","):
            d = _bench(["--force-comm", "--comm-plan", f"peer:shardov:fp32:{b}"])
            meas[d["config"]["comm_plan"]] = [(d["ms_per_step"], d.get("allreduce_ms"))]
        d = _bench(["--force-comm", "--comm-plan", "peer:shardride:fp32:1024"])
        meas[d["config"]["comm_plan"]] = [(d["ms_per_step"], d.get("allreduce_ms"))]
    med = {k: (sorted(x[0] for x in v)[len(v) // 2], max((x[1] or 0.0) for x in v)) for k, v in meas.items()}
    pred = {}
    for N in (2, 4, 8):
        link = 6.0 * (N - 1) / N * N_PARAMS / (a.link_gbs * 1e9) * 1e3          # ms
        row = {}
        for k, (t, span) in med.items():
            if k.startswith("peer:shard:"):
                row[k] = round(t + link, 4)
            elif k.startswith("peer:shardov:"):
                hide = span or 0.0
                row[k] = round(t + FIRST_STAGE_FRAC * link + max(0.0, (1 - FIRST_STAGE_FRAC) * link - hide), 4)
            elif k.startswith("peer:shardride:"):
                f = (N - 1) / N / (a.link_gbs * 1e9) * 1e3                     # ms per byte-count unit
                phases = {"rs_a": 4 * RIDE_A, "rs_b": 4 * RIDE_B, "ag_a": 2 * RIDE_A, "ag_b": 2 * RIDE_B}
                exposed = sum(max(0.0, nb * f - RIDE_WINDOWS_US[p] / 1e3) for p, nb in phases.items())
                rest = 6 * (N_PARAMS - RIDE_A - RIDE_B) * f
                row[k] = round(t + rest + exposed, 4)
        pred[str(N)] = dict(sorted(row.items(), key=lambda kv: kv[1]))
    out = {"measured_world1_ms": {k: v[0] for k, v in med.items()},
           "side_span_world1_ms": {k: v[1] for k, v in med.items() if k.startswith("peer:shardov")},
           "predicted_ms": pred, "link_gbs_assumed": a.link_gbs}
    print(json.dumps(out, indent=1))
    if a.write:
        with open(PLAN) as f:
            plan = json.load(f)
        plan["shard_plans"] = dict(out, source="tools/shard_plan_probe.py")
        for N, row in pred.items():
            best = min(row, key=row.get) if row else None
            shard = next((k for k in row if k.startswith("peer:shard:")), None)
            if best and shard and row[best] < row[shard]:
                plan["choice"][N] = best
        with open(PLAN, "w") as f:
            json.dump(plan, f, indent=1)


if __name__ == "__main__":
    main()
