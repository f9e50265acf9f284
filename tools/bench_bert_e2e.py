"""BERT-base MLM through the whole framework: ``kubeml train -f bert --K 1 --grad-sync`` on one
GPU worker (server, storage, scheduler, parameter server, resident worker), synthetic token ids of
the bench's shape (batch 32 x 512, 76 masked positions per sequence, masked on the device every
step).  Reports the steady per-step time from the job's own epoch logs (train seconds of an epoch
/ its steps, warm-up epochs excluded) next to ``tools/bench_bert.py``'s number when given one.

    python tools/bench_bert_e2e.py [--steps 24] [--epochs 4] [--bench-ms 17.26]
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=24, help="train steps per epoch")
    ap.add_argument("--epochs", type=int, default=4)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--bench-ms", type=float, default=None, help="tools/bench_bert.py ms/step to compare with")
    a = ap.parse_args()
    from kubeml_amd.api.types import TrainOptions, TrainRequest
    from kubeml_amd.client import KubemlClient
    from kubeml_amd.config import Config
    from kubeml_amd.control.server import KubeMLServer
    tmp = tempfile.mkdtemp(prefix="kubeml_bert_e2e_")
    cfg = Config()
    cfg.store_dir = os.path.join(tmp, "store")
    srv = KubeMLServer(cfg, n_workers=1, use_gpu=True, task_timeout=1800).start(
        ports={p: 0 for p in ("controller", "scheduler", "ps", "storage", "metrics")})
    try:
        c = KubemlClient(srv.url())
        rng = np.random.default_rng(0)
        n = a.steps * a.batch
        arrs = {"xtr": rng.integers(1000, 30000, (n, a.seq), dtype=np.int64), "ytr": np.zeros(n, dtype=np.int64),
                "xte": rng.integers(1000, 30000, (a.batch, a.seq), dtype=np.int64),
                "yte": np.zeros(a.batch, dtype=np.int64)}
        paths = {}
        for k, v in arrs.items():
            paths[k] = os.path.join(tmp, f"{k}.npy")
            np.save(paths[k], v)
        c.datasets.create("wiki_tokens", paths["xtr"], paths["ytr"], paths["xte"], paths["yte"])
        c.functions.create("bert", os.path.join(ROOT, "examples", "function_bert.py"))
        t0 = time.time()
        jid = c.networks.train(TrainRequest(batch_size=a.batch, epochs=a.epochs, dataset="wiki_tokens", lr=1e-4,
                                            function_name="bert",
                                            options=TrainOptions(default_parallelism=1, static_parallelism=True,
                                                                 validate_every=0, k=1, sync="grad")))
        last = time.time()
        while c.tasks.status(jid)["state"] == "running":
            time.sleep(0.2)
            if time.time() - last > 30:
                print(f"[bert_e2e] running {time.time() - t0:.0f}s", file=sys.stderr, flush=True)
                last = time.time()
            if time.time() - t0 > 1500:
                raise TimeoutError("bert e2e job did not finish")
        st = c.tasks.status(jid)
        if st["state"] != "finished":
            raise RuntimeError(f"job {jid} {st}: {c.logs(jid).decode()[-3000:]}")
        logs = [json.loads(l) for l in c.logs(jid).decode().splitlines() if l.startswith("{")]
        train_s = [float(l["seconds"]) for l in logs if l.get("msg") == "epoch finished"]
        h = c.histories.get(jid).data
        steady = train_s[2:] if len(train_s) > 2 else train_s[-1:]
        ms = 1e3 * sum(steady) / len(steady) / a.steps
        out = {"metric": "BERT-base MLM step through kubeml train (K=1, grad-sync, 1 GPU worker)",
               "ms_per_step": round(ms, 3), "tokens_per_s": round(a.batch * a.seq / ms * 1e3, 1),
               "epoch_train_s": [round(s, 4) for s in train_s], "steps_per_epoch": a.steps,
               "batch": a.batch, "seq": a.seq, "train_loss": [round(float(x), 4) for x in h.train_loss],
               "sync_mode": list(h.sync_mode), "masking": "device kernel per step (kernels.mlm_mask) inside the graph"}
        if a.bench_ms:
            out["bench_bert_ms"] = a.bench_ms
            out["framework_vs_bench"] = round(ms / a.bench_ms, 4)
        print(json.dumps(out), flush=True)
    finally:
        srv.stop()


if __name__ == "__main__":
    main()
