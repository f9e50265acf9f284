"""BERT-base MLM training throughput on MI355X (north-star config 5; not the headline
bench — see bench.py).  Synthetic token batches of the real shape (there is no network
for a corpus), masked on the device every step (kml_mlm_mask, BERT's 80/10/10 recipe), random-init
BERT-base (109.5 M params), fused AdamW, bf16 compute, fp32 master weights, hidden + attention-probability dropout 0.1, 76 masked positions per
512-token sequence (Google BERT's max_predictions_per_seq), whole step captured as one
hipGraph.  Weight gradients and the GELU-fused FFN2 dgrad run on csrc/kernels/gemm.hip; the
plain forward / dgrad GEMMs (bias or residual addend only) run on hipBLASLt where
``gemm_tuning.json`` says the library measured faster inside the step.

Data parallel (config 5: 8 workers): ``--gpus N`` launches N ranks (one per GPU,
torch.distributed over RCCL/xGMI) unless already under torchrun; backward is split into
3 stages whose gradient ranges are all-reduced while the next stage computes, the
all-reduces captured inside the step graph; AdamW folds in the 1/N average.

    python tools/bench_bert.py [--gpus N] [--batch 32] [--seq 512] [--steps 20] [--warmup 3]
Prints one JSON line on rank 0 (tokens/s over all processed tokens of all ranks).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--preds", type=int, default=76)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--force-comm", action="store_true", help="RCCL path even with one rank (rehearsal)")
    a = ap.parse_args()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        import torch
        if torch.cuda.device_count() < a.gpus:
            print(f"bench_bert: --gpus {a.gpus} but {torch.cuda.device_count()} GPU(s) visible", file=sys.stderr)
            sys.exit(2)
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")))

    import torch
    import torch.distributed as dist
    from kubeml_amd.engine.staged import StagedForwardBackward
    from kubeml_amd.engine.step import GraphedTrainStep, train_state_tensors
    from kubeml_amd.models.bert import BertForMaskedLM
    from kubeml_amd.nn import flatten_module
    from kubeml_amd.optim import AdamW
    from kubeml_amd.parallel.comm import from_env
    from kubeml_amd.parallel.kavg import ModelAverager
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    comm = world > 1 or a.force_comm
    if comm:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29537")
        dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)
    torch.manual_seed(0)
    m = BertForMaskedLM(layers=a.layers, seed=1 + 7919 * rank).to(dev)
    sp = flatten_module(m)
    if comm:
        ModelAverager(m).broadcast_(from_env(), 0)
    m.train()
    opt = AdamW(m.parameters(), lr=1e-4, weight_decay=0.01)
    opt.set_grad_scale(1.0 / world)
    B, L, P, V = a.batch, a.seq, a.preds, 30522
    g = torch.Generator(device=dev).manual_seed(1 + rank)
    raw = torch.randint(0, V, (B, L), device=dev, generator=g)      # the corpus batch (token ids)
    tt = torch.zeros(B, L, dtype=torch.int64, device=dev)
    from kubeml_amd.ops import kernels as K
    ctr = torch.tensor([float(1 + rank), 0.0], dtype=torch.float32, device=dev)
    ids, pos, lab = K.mlm_mask(raw, ctr, P, advance=False)           # static buffers of the step

    def pre():
        # every step masks its batch on the device (a fresh mask per replay), inside the timed region
        K.mlm_mask(raw, ctr, P, out=(ids, pos, lab))
        sp.zero_grad()

    fns, sparams = m.stages(ids, tt, None, pos, lab, n=3)
    staged = StagedForwardBackward(fns, lambda out: out, lambda: ids, pre=pre)
    segs = [staged.segment(k) for k in range(staged.n_segments)]
    seg_grads = [[sp.grad_view(sparams[len(sparams) - 1 - k])] for k in range(len(sparams))]
    step = GraphedTrainStep(None, opt.step, use_graph=not a.no_graph, warmup=1, segments=segs,
                            segment_grads=seg_grads, force_comm=a.force_comm, graph_comm=True,
                            state_tensors=train_state_tensors(m, sp, opt, [m.rng.tensor(dev), ctr]))
    if comm:
        step.prime_comm()
    step.capture()
    for _ in range(a.warmup):
        loss = step()
    torch.cuda.synchronize()
    first = float(loss.detach())
    if comm:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    if comm:
        dist.barrier()
    dt = time.perf_counter() - t0
    in_sync = None
    if comm:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        cs = sp.master.double().abs().sum().view(1)
        lo, hi = cs.clone(), cs.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        in_sync = bool((hi - lo).abs().item() <= 1e-9 * max(1.0, abs(hi.item())))
    tok_s = B * L * world * a.steps / dt
    if rank == 0:
        out = {"metric": "BERT-base MLM training tokens/s (whole job)", "value": round(tok_s, 1), "unit": "tokens/s",
               "n_gpus": world, "ms_per_step": round(dt / a.steps * 1e3, 3), "batch_per_gpu": B, "seq": L,
               "masked_per_seq": P, "masking": "per step on the device (kml_mlm_mask), inside the timed region",
               "layers": a.layers, "optimizer": "fused AdamW", "dtype": "bf16",
               "data": "synthetic tokens, random init", "graph": not a.no_graph, "overlap_segments": len(segs),
               "loss_first_last": [round(first, 4), round(float(loss.detach()), 4)],
               "gemm": "gemm.hip (wgrad, FFN2 dgrad + GELU backward) / hipBLASLt (plain fwd, dgrad: gemm_tuning.json)"}
        if in_sync is not None:
            out["ranks_in_sync"] = in_sync
        print(json.dumps(out), flush=True)
    if comm:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
