"""End-to-end framework benchmark: the headline workload through the whole KubeML stack
(kubeml_amd/experiments/e2e.py: server + GPU workers + storage upload + ``kubeml train``).

Reports, from the job's own history (``epoch_duration`` is cumulative wall time since
training start, reference ml/pkg/train/job.go:327) and log: per-epoch wall time (epoch 1
includes graph capture and warm-up), the steady epoch (mean over epochs >= 2) and the
steady train-task rate, compared with ``bench.py``'s step rate when given (--bench-img-s).

Usage: python tools/bench_e2e.py [--gpus N] [--epochs E] [--validate] [--bench-img-s X] [--trace DIR]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--epochs", type=int, default=4)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--k", type=int, default=1)
    ap.add_argument("--validate", action="store_true", help="validate every epoch (reference time definition)")
    ap.add_argument("--n-train", type=int, default=50000)
    ap.add_argument("--n-test", type=int, default=10000)
    ap.add_argument("--bench-img-s", type=float, default=None)
    ap.add_argument("--function", default=os.path.join(ROOT, "examples", "function_resnet34.py"))
    ap.add_argument("--trace", default=None, help="KUBEML_TRACE=1 in the workers; copy their Chrome traces here")
    a = ap.parse_args()
    if a.trace:
        os.environ["KUBEML_TRACE"] = "1"
    from kubeml_amd.experiments.e2e import run_e2e
    out = {"metric": "end-to-end kubeml train images/s (ResNet-34 CIFAR-10 shape, synthetic)"}
    out.update(run_e2e(gpus=a.gpus, epochs=a.epochs, batch=a.batch, k=a.k, validate=a.validate,
                       n_train=a.n_train, n_test=a.n_test, function=a.function, trace_dir=a.trace,
                       progress=lambda m: print(m, flush=True)))
    if a.bench_img_s:
        out["vs_bench_step_rate"] = round(out["steady_train_task_img_s"] / a.bench_img_s, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
