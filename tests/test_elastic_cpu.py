"""Elastic parallelism and GPU-inventory sharing on CPU workers (gloo).

* A scripted policy forces P = 2 -> 4 -> 2 on a 4-worker node (reference: the
  scheduler changes parallelism between epochs, ml/pkg/scheduler/policy.go:50-94,
  applied at the next fan-out, ml/pkg/train/job.go:196-215).  Per-task model
  checksums show that every active worker ends each epoch with the same model and that
  the workers newly activated at P = 4 STARTED epoch 2 from rank 0's model (the
  epoch-start broadcast over the P-rank sub-communicator).
* Two static jobs with P = 1 on a 2-slot node run concurrently on disjoint slots.
"""
import json
import os
import time

import numpy as np
import pytest

from kubeml_amd.api.types import TrainOptions, TrainRequest
from kubeml_amd.client import KubemlClient
from kubeml_amd.config import Config
from kubeml_amd.control.server import KubeMLServer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PORTS = {k: 0 for k in ("controller", "scheduler", "ps", "storage", "metrics")}


def _data(tmp, n=1280, seed=0):
    from tests.test_control_cpu import mnist_like
    xtr, ytr = mnist_like(n, seed)
    xte, yte = mnist_like(256, seed + 1)
    paths = {}
    for name, arr in (("xtr", xtr), ("ytr", ytr), ("xte", xte), ("yte", yte)):
        paths[name] = os.path.join(tmp, name + ".npy")
        np.save(paths[name], arr)
    return paths


def _wait(c, jid, timeout=300):
    t0 = time.time()
    while time.time() - t0 < timeout:
        st = c.tasks.status(jid)
        if st["state"] != "running":
            return st
        time.sleep(0.2)
    raise TimeoutError(jid)


def _epoch_logs(c, jid):
    recs = [json.loads(l) for l in c.logs(jid).decode().splitlines() if l.startswith("{")]
    return [r for r in recs if r.get("msg") == "epoch finished"]


def test_scripted_resize_2_4_2_keeps_workers_consistent(tmp_path):
    cfg = Config()
    cfg.store_dir = str(tmp_path / "store")
    srv = KubeMLServer(cfg, n_workers=4, use_gpu=False, task_timeout=300, policy="scripted:2,4,2").start(ports=PORTS)
    try:
        c = KubemlClient(srv.url())
        p = _data(str(tmp_path))
        c.datasets.create("mnist", p["xtr"], p["ytr"], p["xte"], p["yte"])
        c.functions.create("lenet", os.path.join(ROOT, "examples", "function_lenet.py"))
        jid = c.networks.train(TrainRequest(batch_size=64, epochs=3, dataset="mnist", lr=0.05, function_name="lenet",
                                            options=TrainOptions(default_parallelism=2, static_parallelism=False,
                                                                 validate_every=0, k=2)))
        st = _wait(c, jid)
        assert st["state"] == "finished", (st, c.logs(jid).decode()[-3000:])
        h = c.histories.get(jid).data
        assert h.parallelism == [2.0, 4.0, 2.0]
        eps = _epoch_logs(c, jid)
        assert [len(e["checksums"]) for e in eps] == [2, 4, 2]
        prev_end = None
        for e in eps:
            ck = {int(r): v for r, v in e["checksums"].items()}
            starts = [v[0] for v in ck.values()]
            ends = [v[1] for v in ck.values()]
            # all active workers start from one model ...
            assert max(starts) - min(starts) <= 1e-9 * max(1.0, abs(starts[0])), e["checksums"]
            # ... which is the model the previous epoch ended with (new ranks got rank 0's)
            if prev_end is not None:
                assert abs(starts[0] - prev_end) <= 1e-9 * max(1.0, abs(prev_end)), (starts, prev_end)
            assert max(ends) - min(ends) <= 1e-6 * max(1.0, abs(ends[0])), e["checksums"]
            assert ends[0] != starts[0]
            prev_end = ends[0]
    finally:
        srv.stop()


def test_two_static_jobs_share_the_node(tmp_path):
    cfg = Config()
    cfg.store_dir = str(tmp_path / "store")
    srv = KubeMLServer(cfg, n_workers=2, use_gpu=False, task_timeout=300).start(ports=PORTS)
    try:
        c = KubemlClient(srv.url())
        p = _data(str(tmp_path), n=2560)
        c.datasets.create("mnist", p["xtr"], p["ytr"], p["xte"], p["yte"])
        c.functions.create("lenet", os.path.join(ROOT, "examples", "function_lenet.py"))
        req = TrainRequest(batch_size=16, epochs=2, dataset="mnist", lr=0.02, function_name="lenet",
                           options=TrainOptions(default_parallelism=1, static_parallelism=True, k=-1))
        j1 = c.networks.train(req)
        j2 = c.networks.train(req)
        both = False
        t0 = time.time()
        while time.time() - t0 < 120:
            alloc = dict(srv.ps.alloc)
            if j1 in alloc and j2 in alloc:
                both = True
                assert set(alloc[j1]).isdisjoint(alloc[j2]) and len(alloc[j1]) == len(alloc[j2]) == 1
                break
            time.sleep(0.05)
        assert both, "the second static job did not get its own slot"
        for j in (j1, j2):
            assert _wait(c, j)["state"] == "finished"
    finally:
        srv.stop()


def test_non_fp32_buffers_are_averaged_by_the_side_pack():
    """Buffers outside the fp32 state (fp64, int32, bool, non-scalar int64) are averaged with
    the reference's rules (floats averaged, integers floor-divided) and broadcast."""
    import threading

    import torch
    from kubeml_amd.nn.flat import flatten_module
    from kubeml_amd.parallel.comm import ThreadComm
    from kubeml_amd.parallel.kavg import ModelAverager

    class Odd(torch.nn.Module):
        def __init__(self, r):
            super().__init__()
            self.lin = torch.nn.Linear(2, 2)
            self.register_buffer("f64", torch.full((3,), float(r), dtype=torch.float64))
            self.register_buffer("i32", torch.full((2,), 3 * r + 1, dtype=torch.int32))
            self.register_buffer("vec64", torch.tensor([r, 2 * r], dtype=torch.int64))

    world = 3
    comms = ThreadComm.create(world)
    mods = [Odd(r) for r in range(world)]
    for m in mods:
        flatten_module(m)
        assert {n for _, n in m._kml_flat.other_buffers} == {"f64", "i32", "vec64"}

    def body(r):
        av = ModelAverager(mods[r])
        av._average_other(comms[r], mods[r]._kml_flat, True)
    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(30)
    for m in mods:
        assert m.f64.dtype == torch.float64 and torch.allclose(m.f64, torch.full((3,), 1.0, dtype=torch.float64))
        assert m.i32.dtype == torch.int32 and m.i32.tolist() == [4, 4]          # floor((1+4+7)/3)
        assert m.vec64.tolist() == [1, 2]                                         # floor(3/3), floor(6/3)
