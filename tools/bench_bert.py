"""BERT-base MLM training throughput on MI355X (north-star config 5; not the headline
bench — see bench.py).  Synthetic token batches of the real shape (there is no
network for a corpus), random-init BERT-base (109.5 M params), AdamW, bf16 compute,
fp32 master weights, hidden dropout 0.1, 76 masked positions per 512-token sequence
(Google BERT's max_predictions_per_seq), whole step captured as one hipGraph.

    python tools/bench_bert.py [--batch 32] [--seq 512] [--steps 20] [--warmup 3]
Prints one JSON line (tokens/s over all processed tokens).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--preds", type=int, default=76)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--no-graph", action="store_true")
    a = ap.parse_args()
    import torch
    from kubeml_amd.engine.step import GraphedTrainStep
    from kubeml_amd.models.bert import BertForMaskedLM
    from kubeml_amd.nn import flatten_module
    from kubeml_amd.optim import AdamW
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = BertForMaskedLM(layers=a.layers).to(dev)
    sp = flatten_module(m)
    m.train()
    opt = AdamW(m.parameters(), lr=1e-4, weight_decay=0.01)
    B, L, P, V = a.batch, a.seq, a.preds, 30522
    g = torch.Generator(device=dev).manual_seed(1)
    ids = torch.randint(0, V, (B, L), device=dev, generator=g)
    tt = torch.zeros(B, L, dtype=torch.int64, device=dev)
    pos = torch.stack([torch.randperm(L, device=dev, generator=g)[:P].sort().values for _ in range(B)])
    lab = torch.randint(0, V, (B, P), device=dev, generator=g)

    def fb():
        sp.zero_grad()
        loss = m(ids, tt, None, pos, lab)
        loss.backward()
        return loss
    step = GraphedTrainStep(fb, opt.step, use_graph=not a.no_graph, warmup=2)
    step.capture()
    for _ in range(a.warmup):
        loss = step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ms = dt / a.steps * 1e3
    tok = B * L * a.steps / dt
    # model FLOPs: 6 * params(non-embedding) * tokens + attention 12*L*d*layers*tokens, plus the MLM head
    d, I, nl = 768, 3072, a.layers
    dense = 6 * B * L * nl * (4 * d * d + 2 * d * I) + 6 * B * L * nl * 2 * L * d
    head = 6 * B * P * (d * d + d * V)
    tflops = (dense + head) / (ms / 1e3) / 1e12
    print(json.dumps({"metric": "BERT-base MLM training tokens/s (1 GPU)", "value": round(tok, 1), "unit": "tokens/s",
                      "ms_per_step": round(ms, 3), "batch": B, "seq_len": L, "masked_per_seq": P,
                      "layers": nl, "dtype": "bf16", "optimizer": "AdamW", "model_tflops": round(tflops, 1),
                      "loss": round(float(loss), 4), "graph": not a.no_graph,
                      "data": "synthetic tokens, random init"}), flush=True)


if __name__ == "__main__":
    main()
