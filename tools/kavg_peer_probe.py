"""Time one K-AVG round on the ResNet-34 flat state: fused peer round (comm.hip kml_peer_kavg)
vs the unfused pair (peer two-shot all-reduce + kml_kavg_finish), N ranks packed on one GPU.

Packed ranks share one HBM, so this measures the kernels' memory passes, not xGMI: it shows
what the fusion removes (the finish pass over the whole state) and that nothing else grew.

    python tools/kavg_peer_probe.py [--world 2] [--rounds 20]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def _run(rank, world, port, rounds, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from kubeml_amd.models.resnet import resnet34
        from kubeml_amd.nn import flatten_module
        from kubeml_amd.ops import kernels as K
        from kubeml_amd.parallel.peer import PeerAllReduce, slot_bytes
        net = resnet34(10).to(dev)
        sp = flatten_module(net)
        arena = sp.i64_arena_now()
        ar = PeerAllReduce(None, cap_bytes=slot_bytes(sp.state.numel(), world, "twoshot"), device=dev)

        def fused():
            K.kavg_pack_(sp.state, arena, sp.i64_off, sp.n_i64, sp.count_idx, True)
            ar.kavg_(sp.state, sp.count_idx, sp.numel, sp.shadow, arena, sp.i64_off, sp.n_i64)

        def unfused():
            K.kavg_pack_(sp.state, arena, sp.i64_off, sp.n_i64, sp.count_idx, True)
            ar.all_reduce_(sp.state, algo="twoshot")
            K.kavg_finish_(sp.state, sp.numel, sp.count_idx, sp.shadow, arena, sp.i64_off, sp.n_i64)

        out = {"state_mb": round(sp.state.numel() * 4 / 1e6, 1), "world": world}
        for name, fn in (("unfused_ms", unfused), ("fused_ms", fused), ("unfused_ms_2", unfused),
                         ("fused_ms_2", fused)):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            dist.barrier()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(rounds):
                fn()
            e1.record()
            torch.cuda.synchronize()
            out[name] = round(e0.elapsed_time(e1) / rounds, 3)
        ar.check()
        dist.barrier()
        ar.close()
        q.put((rank, out, None))
    except Exception as e:
        q.put((rank, None, repr(e)))
    finally:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=20)
    a = ap.parse_args()
    import torch.multiprocessing as mp
    from kubeml_amd.runtime.pool import free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_run, args=(r, a.world, port, a.rounds, q)) for r in range(a.world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(30)
    for rank, out, err in res:
        if err:
            raise SystemExit(f"rank {rank}: {err}")
    print(json.dumps({"ranks": [r[1] for r in res]}))


if __name__ == "__main__":
    main()
