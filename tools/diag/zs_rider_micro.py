"""Shard-rider slices launched on their own (one rank, ResNet-34's flat space): per-slice time of
the reduce-scatter + fused SGD rider (``ShardRider.run_alone``) against the plain ranged SGD over
the same elements, for several rider block counts.  Isolates the rider code path from the conv
launches that normally host it (engine/dp.py ``shardride``).

    python tools/diag/zs_rider_micro.py [--reps 20]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    dist.init_process_group("gloo", rank=0, world_size=1)
    from kubeml_amd.models.resnet import resnet34
    from kubeml_amd.nn import flatten_module
    from kubeml_amd.optim import SGD
    from kubeml_amd.parallel.peer import PeerShard
    dev = torch.device("cuda", 0)
    model = resnet34(num_classes=1000).to(dev)
    space = flatten_module(model)
    opt = SGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    space.grad.normal_()
    space.sync_master()
    sh = PeerShard(space)
    groups = model.comm_ride_plan()
    ranges = [space.range_of(ps) for ps, _, _ in groups]
    sh.set_stages([ranges[0], ranges[1], (ranges[1][1], space.numel)])

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1000.0 / a.reps
    for gi, (ps, rs_hosts, _) in enumerate(groups):
        lo, hi = ranges[gi]
        t_sgd = timeit(lambda: opt.step_range(lo, hi, advance_step=False))
        for blocks in (128, 256, 512, 1024):
            sl = sh.rider_slices(gi, "rs", len(rs_hosts), opt, blocks)

            def run():
                for r in sl:
                    r.run_alone()
            t = timeit(run)
            one = timeit(lambda: sl[0].run_alone())
            print(json.dumps({"stage": gi, "elements": hi - lo, "slices": len(sl), "blocks": blocks,
                              "rider_all_us": round(t, 1), "rider_one_slice_us": round(one, 2),
                              "plain_sgd_us": round(t_sgd, 1)}), flush=True)
    sh.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
