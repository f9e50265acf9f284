"""``kubeml`` command line — same subcommands and flags as the reference's cobra CLI
(ml/pkg/kubeml-cli/cmd/*.go):

  train     -d/--dataset -f/--function -e/--epochs(1) -b/--batch(64) --lr(0.01)
            --validate-every(0) --parallelism(2) --static --K(-1) --sparse-avg
            --goal-accuracy(100)        [alias: --default-parallelism]
  dataset   create -n --traindata --trainlabels --testdata --testlabels | delete -n | list
  function|fn  create --name --code | delete --name | list
  task      list [--short] | stop --id | prune
  history   get --id | delete --id | list | prune        [alias: --network for --id]
  infer     -n/--network --datafile
  logs      --id [-f/--follow]
  server    start the single-node control plane (kubeml-server)

Extras: ``train --wait`` blocks until the job finishes and prints its history.
The controller URL is ``KUBEML_CONTROLLER_URL`` (default http://127.0.0.1:10100).
"""
from __future__ import annotations

import argparse
import json
import math
import sys
import time
from typing import List, Optional

from .api.errors import KubeMLException
from .api.types import MAX_BATCH, InferRequest, TrainOptions, TrainRequest


def _client(args):
    from .client import KubemlClient
    return KubemlClient(getattr(args, "url", None))


def _table(rows: List[List], out=sys.stdout):
    """tabwriter(minwidth 1, tabwidth 1, padding 2) look-alike."""
    if not rows:
        return
    w = [max(len(str(r[i])) for r in rows) for i in range(len(rows[0]))]
    for r in rows:
        out.write("".join(str(c).ljust(w[i] + 2) if i < len(r) - 1 else str(c) for i, c in enumerate(r)).rstrip()
                  + "\n")


def _last(xs):
    return xs[-1] if xs else math.nan


def _mean(xs):
    return sum(xs) / len(xs) if xs else math.nan


def _confirm(prompt: str, yes: bool) -> bool:
    if yes:
        return True
    try:
        return input(f"{prompt} [y/N]: ").strip().lower() in ("y", "yes")
    except EOFError:
        return False


# ------------------------------------------------------------------------------ train
def cmd_train(a):
    c = _client(a)
    K = -1 if a.sparse_avg else a.K
    req = TrainRequest(model_type="example", batch_size=a.batch, epochs=a.epochs, dataset=a.dataset, lr=a.lr,
                       function_name=a.function,
                       options=TrainOptions(default_parallelism=a.parallelism, static_parallelism=a.static,
                                            validate_every=a.validate_every, k=K, goal_accuracy=a.goal_accuracy,
                                            resume_from=a.resume or "", sync="grad" if a.grad_sync else ""))
    # validateTrainRequest (train.go:150-172)
    if not (0 < req.batch_size <= MAX_BATCH):
        raise KubeMLException(f"batch size must be between 1 and {MAX_BATCH}", 400)
    if req.epochs <= 0:
        raise KubeMLException("epochs must be positive", 400)
    if req.lr <= 0:
        raise KubeMLException("learning rate must be positive", 400)
    if req.options.sync == "grad" and req.options.k != 1:
        raise KubeMLException("--grad-sync runs K = 1 rounds: pass --K 1", 400)
    if req.options.sync == "grad" and not req.options.static_parallelism:
        # the optimizer state persists across rounds and lives sharded per rank: a resize would
        # leave new workers with zero moments and hand chunks to stale owners
        raise KubeMLException("--grad-sync keeps optimizer state on the workers: pass --static", 400)
    c.datasets.get(req.dataset)
    if not any(f["name"] == req.function_name for f in c.functions.list()):
        raise KubeMLException(f"function {req.function_name} does not exist", 404)
    jid = c.networks.train(req)
    print(jid)
    if a.wait:
        while True:
            st = c.tasks.status(jid)
            if st["state"] != "running":
                break
            time.sleep(0.5)
        if st.get("error"):
            raise KubeMLException(f"job {jid} failed: {st['error']}", 500)
        print(json.dumps(c.histories.get(jid).to_dict(), indent=2))


# ------------------------------------------------------------------------------ dataset
def cmd_dataset_create(a):
    r = _client(a).datasets.create(a.name, a.traindata, a.trainlabels, a.testdata, a.testlabels)
    print(r.get("result", r) if isinstance(r, dict) else r)


def cmd_dataset_delete(a):
    r = _client(a).datasets.delete(a.name)
    print(r.get("result", r) if isinstance(r, dict) else r)


def cmd_dataset_list(a):
    rows = [["NAME", "TRAINSET", "TESTSET"]]
    for d in _client(a).datasets.list():
        rows.append([d.name, d.train_set_size, d.test_set_size])
    _table(rows)


# ------------------------------------------------------------------------------ function
def cmd_fn_create(a):
    _client(a).functions.create(a.name, a.code)
    print(f"function {a.name} created")


def cmd_fn_delete(a):
    _client(a).functions.delete(a.name)
    print(f"function {a.name} deleted")


def cmd_fn_list(a):
    rows = [["NAME", "ENVIRONMENT", "CONCURRENCY", "TIMEOUT", "CREATED"]]
    for f in _client(a).functions.list():
        rows.append([f["name"], f["environment"], f["concurrency"], f["timeout"],
                     time.strftime("%Y-%m-%dT%H:%M:%S", time.localtime(f["created"]))])
    _table(rows)


# ------------------------------------------------------------------------------ task
def cmd_task_list(a):
    tasks = _client(a).tasks.list()
    if a.short:
        for t in tasks:
            print(t.job.id)
        return
    rows = [["NAME", "FUNCTION", "DATASET", "MODEL", "EPOCHS", "BATCH", "LR"]]
    for t in tasks:
        r = t.request
        rows.append([t.job.id, r.function_name, r.dataset, r.model_type, r.epochs, r.batch_size, r.lr])
    _table(rows)


def cmd_task_stop(a):
    _client(a).tasks.stop(a.id)
    print(f"task {a.id} stopped")


def cmd_task_prune(a):
    """reference deletes leftover job pods/services; here: stop every running task."""
    c = _client(a)
    if not _confirm("This will stop every running task. Continue?", a.yes):
        return
    for t in c.tasks.list():
        c.tasks.stop(t.job.id)
        print(f"stopped {t.job.id}")


# ------------------------------------------------------------------------------ history
def cmd_history_get(a):
    print(json.dumps(_client(a).histories.get(a.id).to_dict(), indent=2))


def cmd_history_delete(a):
    _client(a).histories.delete(a.id)
    print(f"history {a.id} deleted")


def cmd_history_list(a):
    rows = [["NAME", "MODEL", "DATASET", "EPOCHS", "BATCH", "LR", "PARALLELISM", "K", "STATIC", "ACCURACY", "LOSS",
             "TIME (s)"]]
    for h in _client(a).histories.list():
        t, d = h.task, h.data
        rows.append([h.id, t.model_type, t.dataset, t.epochs, t.batch_size, t.lr, _mean(d.parallelism),
                     t.options.k, str(t.options.static_parallelism).lower(), _last(d.accuracy),
                     _last(d.validation_loss), _last(d.epoch_duration)])
    _table(rows)


def cmd_history_prune(a):
    if not _confirm("This will delete every training history. Continue?", a.yes):
        return
    _client(a).histories.prune()
    print("histories pruned")


# ------------------------------------------------------------------------------ infer / logs
def cmd_infer(a):
    with open(a.datafile) as f:
        data = json.load(f)
    if not isinstance(data, list):
        raise KubeMLException("datafile must hold a JSON array", 400)
    print(json.dumps(_client(a).networks.infer(InferRequest(model_id=a.network, data=data))))


def cmd_logs(a):
    c = _client(a)
    off = 0
    while True:
        chunk = c.logs(a.id, off)
        if chunk:
            sys.stdout.write(chunk.decode(errors="replace"))
            sys.stdout.flush()
            off += len(chunk)
        if not a.follow:
            return
        try:
            if c.tasks.status(a.id)["state"] != "running":
                chunk = c.logs(a.id, off)
                sys.stdout.write(chunk.decode(errors="replace"))
                return
        except KubeMLException:
            return
        time.sleep(1.0)


def cmd_server(a):
    from .control.server import main as server_main
    argv = []
    if a.store:
        argv += ["--store", a.store]
    if a.workers is not None:
        argv += ["--workers", str(a.workers)]
    if a.cpu:
        argv += ["--cpu"]
    server_main(argv)


# ------------------------------------------------------------------------------ parser
def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser("kubeml", description="KubeML on MI355X")
    p.add_argument("--url", default=None, help="controller URL (KUBEML_CONTROLLER_URL)")
    sub = p.add_subparsers(dest="cmd", required=True)

    t = sub.add_parser("train", help="train a network")
    t.add_argument("-d", "--dataset", required=True)
    t.add_argument("-f", "--function", required=True)
    t.add_argument("-e", "--epochs", type=int, default=1)
    t.add_argument("-b", "--batch", type=int, default=64)
    t.add_argument("--lr", type=float, default=0.01)
    t.add_argument("--validate-every", type=int, default=0)
    t.add_argument("--parallelism", "--default-parallelism", dest="parallelism", type=int, default=2)
    t.add_argument("--static", action="store_true")
    t.add_argument("--K", "-K", dest="K", type=int, default=-1)
    t.add_argument("--sparse-avg", action="store_true")
    t.add_argument("--goal-accuracy", type=float, default=100.0)
    t.add_argument("--wait", action="store_true", help="block until the job ends, print its history")
    t.add_argument("--resume", default=None, help="continue from the checkpoint/history of this job id")
    t.add_argument("--grad-sync", action="store_true",
                   help="K=1 as synchronous data parallelism with persistent optimizer state (any fused "
                        "optimizer, e.g. AdamW); default: the reference's per-round optimizer reset")
    t.set_defaults(fn=cmd_train)

    d = sub.add_parser("dataset", help="manage datasets").add_subparsers(dest="sub", required=True)
    dc = d.add_parser("create")
    dc.add_argument("-n", "--name", required=True)
    dc.add_argument("--traindata", required=True)
    dc.add_argument("--trainlabels", required=True)
    dc.add_argument("--testdata", required=True)
    dc.add_argument("--testlabels", required=True)
    dc.set_defaults(fn=cmd_dataset_create)
    dd = d.add_parser("delete")
    dd.add_argument("-n", "--name", required=True)
    dd.set_defaults(fn=cmd_dataset_delete)
    d.add_parser("list").set_defaults(fn=cmd_dataset_list)

    for name in ("function", "fn"):
        f = sub.add_parser(name, help="manage functions").add_subparsers(dest="sub", required=True)
        fc = f.add_parser("create")
        fc.add_argument("--name", required=True)
        fc.add_argument("--code", required=True)
        fc.set_defaults(fn=cmd_fn_create)
        fd = f.add_parser("delete")
        fd.add_argument("--name", required=True)
        fd.set_defaults(fn=cmd_fn_delete)
        f.add_parser("list").set_defaults(fn=cmd_fn_list)

    tk = sub.add_parser("task", help="manage tasks").add_subparsers(dest="sub", required=True)
    tl = tk.add_parser("list")
    tl.add_argument("--short", action="store_true")
    tl.set_defaults(fn=cmd_task_list)
    ts = tk.add_parser("stop")
    ts.add_argument("--id", required=True)
    ts.set_defaults(fn=cmd_task_stop)
    tp = tk.add_parser("prune")
    tp.add_argument("-y", "--yes", action="store_true")
    tp.set_defaults(fn=cmd_task_prune)

    h = sub.add_parser("history", help="training histories").add_subparsers(dest="sub", required=True)
    hg = h.add_parser("get")
    hg.add_argument("--id", "--network", dest="id", required=True)
    hg.set_defaults(fn=cmd_history_get)
    hd = h.add_parser("delete")
    hd.add_argument("--id", "--network", dest="id", required=True)
    hd.set_defaults(fn=cmd_history_delete)
    h.add_parser("list").set_defaults(fn=cmd_history_list)
    hp = h.add_parser("prune")
    hp.add_argument("-y", "--yes", action="store_true")
    hp.set_defaults(fn=cmd_history_prune)

    i = sub.add_parser("infer", help="run inference with a trained network")
    i.add_argument("-n", "--network", required=True)
    i.add_argument("--datafile", required=True)
    i.set_defaults(fn=cmd_infer)

    lg = sub.add_parser("logs", help="logs of a job")
    lg.add_argument("--id", required=True)
    lg.add_argument("-f", "--follow", action="store_true")
    lg.set_defaults(fn=cmd_logs)

    sv = sub.add_parser("server", help="start the single-node control plane")
    sv.add_argument("--store", default=None)
    sv.add_argument("--workers", type=int, default=None)
    sv.add_argument("--cpu", action="store_true")
    sv.set_defaults(fn=cmd_server)
    return p


def main(argv: Optional[List[str]] = None) -> int:
    a = build_parser().parse_args(argv)
    try:
        a.fn(a)
    except KubeMLException as e:
        print(f"Error: {e.message}", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
