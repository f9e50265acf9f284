"""End-to-end control plane on CPU workers (north-star config 1: LeNet / MNIST-shaped).

Starts the single-node server (controller, scheduler, PS, storage, metrics on
ephemeral ports) with 2 CPU worker processes (gloo), then drives it over HTTP with the
client library exactly like the CLI does: dataset create, function create, train
(K-AVG, elastic policy, validation), history, metrics, tasks, infer, logs, error paths.
"""
import json
import os
import time

import numpy as np
import pytest

from kubeml_amd.api.types import InferRequest, TrainOptions, TrainRequest
from kubeml_amd.client import KubemlClient
from kubeml_amd.config import Config
from kubeml_amd.control.http import HttpError
from kubeml_amd.control.server import KubeMLServer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PORTS = {k: 0 for k in ("controller", "scheduler", "ps", "storage", "metrics")}


def mnist_like(n, seed):
    """Learnable synthetic MNIST: class k = bright 6x6 block at a class-specific spot."""
    rng = np.random.default_rng(seed)
    y = rng.integers(0, 10, n).astype(np.int64)
    x = rng.integers(0, 40, (n, 28, 28)).astype(np.uint8)
    for i, k in enumerate(y):
        r, c = 2 + (k // 5) * 12, 2 + (k % 5) * 5
        x[i, r:r + 6, c:c + 5] = 250
    return x, y


def _write_dataset(d):
    xtr, ytr = mnist_like(1280, 0)
    xte, yte = mnist_like(256, 1)
    paths = {}
    for name, arr in (("xtr", xtr), ("ytr", ytr), ("xte", xte), ("yte", yte)):
        paths[name] = os.path.join(d, name + ".npy")
        np.save(paths[name], arr)
    return paths, xte


def _start(tmp_path, **kw):
    cfg = Config()
    cfg.store_dir = str(tmp_path / "store")
    srv = KubeMLServer(cfg, n_workers=2, use_gpu=False, task_timeout=300, **kw).start(ports=PORTS)
    return srv, KubemlClient(srv.url())


def _wait(c, jid, timeout=300):
    t0 = time.time()
    while time.time() - t0 < timeout:
        st = c.tasks.status(jid)
        if st["state"] != "running":
            return st
        time.sleep(0.2)
    raise TimeoutError(jid)


@pytest.fixture(scope="module")
def env(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("e2e")
    srv, c = _start(tmp)
    paths, xte = _write_dataset(str(tmp))
    c.datasets.create("mnist", paths["xtr"], paths["ytr"], paths["xte"], paths["yte"])
    c.functions.create("lenet", os.path.join(ROOT, "examples", "function_lenet.py"))
    yield srv, c, xte
    srv.stop()


def test_dataset_and_function_registry(env):
    srv, c, _ = env
    s = c.datasets.get("mnist")
    assert (s.name, s.train_set_size, s.test_set_size) == ("mnist", 1200, 200)  # reference rounding
    assert [d.name for d in c.datasets.list()] == ["mnist"]
    assert [f["name"] for f in c.functions.list()] == ["lenet"]
    with pytest.raises(HttpError) as e:
        c.datasets.get("nope")
    assert e.value.status_code == 404


def test_train_validate_history_infer(env):
    srv, c, xte = env
    req = TrainRequest(batch_size=64, epochs=3, dataset="mnist", lr=0.05, function_name="lenet",
                       options=TrainOptions(default_parallelism=2, static_parallelism=False, validate_every=1, k=4,
                                            goal_accuracy=100))
    jid = c.networks.train(req)
    assert len(jid) == 8
    st = _wait(c, jid)
    assert st["state"] == "finished", st
    h = c.histories.get(jid)
    d = h.data
    assert len(d.train_loss) == 3 and len(d.parallelism) == 3 and len(d.epoch_duration) == 3
    assert d.epoch_duration == sorted(d.epoch_duration)          # cumulative (job.go:327)
    assert len(d.accuracy) == 3 and len(d.validation_loss) == 3  # epochs 1,2 + final
    assert all(1 <= p <= 2 for p in d.parallelism)
    assert d.train_loss[-1] < d.train_loss[0]
    assert d.accuracy[-1] > 30.0, d.accuracy
    assert h.task.function_name == "lenet"
    # checkpoint -> inference works (the reference's infer never loaded weights)
    preds = c.networks.infer(InferRequest(model_id=jid, data=(xte[:4].astype(np.float32) / 255.0).tolist()))
    preds = preds["predictions"]  # the function's response envelope (network.py:154-168)
    assert len(preds) == 4 and all(isinstance(p, int) for p in preds)
    # logs, metrics
    log = c.logs(jid).decode()
    assert "epoch finished" in log and "training finished" in log
    from kubeml_amd.control.http import call
    m = call("GET", srv.url("metrics") + "/metrics")
    assert "kubeml_job_running_total" in m
    # history list / delete
    assert jid in [x.id for x in c.histories.list()]


def test_allreduce_seconds_exported_while_a_two_worker_job_runs(env):
    """K-AVG rounds of a 2-worker job are timed on the workers (sync_seconds per epoch) and
    the PS exports them as kubeml_allreduce_seconds{jobid} while the job runs."""
    import re
    from kubeml_amd.control.http import call
    srv, c, _ = env
    req = TrainRequest(batch_size=32, epochs=6, dataset="mnist", lr=0.05, function_name="lenet",
                       options=TrainOptions(default_parallelism=2, static_parallelism=True, validate_every=0, k=2,
                                            goal_accuracy=100))
    jid = c.networks.train(req)
    pat = re.compile(r'kubeml_allreduce_seconds\{jobid="%s"\} ([0-9.e+-]+)' % jid)
    seen, t0 = [], time.time()
    while c.tasks.status(jid)["state"] == "running" and time.time() - t0 < 300:
        m = call("GET", srv.url("metrics") + "/metrics")
        m = m.decode() if isinstance(m, bytes) else str(m)
        seen += [float(v) for v in pat.findall(m)]
        time.sleep(0.02)
    assert c.tasks.status(jid)["state"] == "finished"
    ep = [json.loads(l) for l in c.logs(jid).decode().splitlines()
          if l.startswith("{") and '"epoch finished"' in l]
    assert ep and all(float(e.get("sync_seconds") or 0) > 0 for e in ep), ep
    assert any(v > 0 for v in seen), seen


def test_job_rest_surface_through_ps(env):
    """The TrainJob's own routes (reference ml/pkg/train/api.go) are served via the PS:
    /job/{id}/status while the job runs, 404 for an unknown job."""
    import time
    from kubeml_amd.control.http import call
    srv, c, _ = env
    req = TrainRequest(batch_size=64, epochs=4, dataset="mnist", lr=0.05, function_name="lenet",
                       options=TrainOptions(default_parallelism=1, static_parallelism=True, validate_every=0, k=4,
                                            goal_accuracy=100))
    jid = c.networks.train(req)
    st, t0 = None, time.time()
    while time.time() - t0 < 60:
        try:
            st = call("GET", srv.url("ps") + f"/job/{jid}/status")
            break
        except HttpError:
            time.sleep(0.05)
    assert st is not None and st["id"] == jid and st["parallelism"] == 1, st
    assert call("GET", srv.url("ps") + f"/job/{jid}/health") in ("", b"", None)
    with pytest.raises(HttpError) as e:
        call("GET", srv.url("ps") + "/job/nosuchjob/status")
    assert e.value.status_code == 404
    assert _wait(c, jid)["state"] == "finished"


def test_request_validation_errors(env):
    srv, c, _ = env
    with pytest.raises(HttpError) as e:
        c.networks.train(TrainRequest(batch_size=4096, epochs=1, dataset="mnist", lr=0.1, function_name="lenet"))
    assert e.value.status_code == 400
    with pytest.raises(HttpError) as e:
        c.networks.train(TrainRequest(batch_size=64, epochs=1, dataset="missing", lr=0.1, function_name="lenet"))
    assert e.value.status_code == 404
    with pytest.raises(HttpError) as e:
        c.networks.train(TrainRequest(batch_size=64, epochs=1, dataset="mnist", lr=0.1, function_name="nofn"))
    assert e.value.status_code == 404
    # persistent (sharded) optimizer state needs a fixed worker group and K = 1
    for opts in (TrainOptions(k=1, sync="grad"), TrainOptions(k=4, static_parallelism=True, sync="grad")):
        with pytest.raises(HttpError) as e:
            c.networks.train(TrainRequest(batch_size=64, epochs=1, dataset="mnist", lr=0.1, function_name="lenet",
                                          options=opts))
        assert e.value.status_code == 400


def test_stop_task(env):
    srv, c, _ = env
    req = TrainRequest(batch_size=16, epochs=50, dataset="mnist", lr=0.01, function_name="lenet",
                       options=TrainOptions(default_parallelism=2, static_parallelism=True, k=-1))
    jid = c.networks.train(req)
    t0 = time.time()
    while not any(t.job.id == jid for t in c.tasks.list()):
        assert time.time() - t0 < 60
        time.sleep(0.1)
    c.tasks.stop(jid)
    st = _wait(c, jid)
    assert st["state"] == "failed" and "force stopped" in st["error"]
    assert len(c.histories.get(jid).data.train_loss) < 50


def test_worker_loss_recovery(tmp_path):
    """KUBEML_FAULT kills rank 1 in epoch 1, round 1: the job rebuilds its pool on the
    survivor, restores the post-init checkpoint and finishes with parallelism 1."""
    srv, c = _start(tmp_path, worker_env={"KUBEML_FAULT": "kill:at=round:rank=1:epoch=1:round=1"})
    try:
        paths, _ = _write_dataset(str(tmp_path))
        c.datasets.create("mnist", paths["xtr"], paths["ytr"], paths["xte"], paths["yte"])
        c.functions.create("lenet", os.path.join(ROOT, "examples", "function_lenet.py"))
        req = TrainRequest(batch_size=64, epochs=2, dataset="mnist", lr=0.05, function_name="lenet",
                           options=TrainOptions(default_parallelism=2, static_parallelism=True, k=2))
        jid = c.networks.train(req)
        st = _wait(c, jid)
        assert st["state"] == "finished", st
        h = c.histories.get(jid).data
        assert h.parallelism == [1.0, 1.0]
        log = c.logs(jid).decode()
        assert "recovering" in log
    finally:
        srv.stop()


def test_hung_worker_detected_and_recovered(tmp_path):
    """KUBEML_FAULT hangs rank 1 at epoch 1, round 2 (alive but stuck; its peer waits in the
    round's all-reduce): no rank makes progress for KUBEML_STALL_TIMEOUT, the pool aborts
    the task (hung collective, culprit = the rank behind) long before the task timeout, and
    the job recovers on the survivor."""
    srv, c = _start(tmp_path, worker_env={"KUBEML_FAULT": "hang:at=round:rank=1:epoch=1:round=2:secs=600"})
    import kubeml_amd.runtime.pool as P
    old = os.environ.get("KUBEML_STALL_TIMEOUT")
    os.environ["KUBEML_STALL_TIMEOUT"] = "4"
    try:
        paths, _ = _write_dataset(str(tmp_path))
        c.datasets.create("mnist", paths["xtr"], paths["ytr"], paths["xte"], paths["yte"])
        c.functions.create("lenet", os.path.join(ROOT, "examples", "function_lenet.py"))
        req = TrainRequest(batch_size=64, epochs=1, dataset="mnist", lr=0.05, function_name="lenet",
                           options=TrainOptions(default_parallelism=2, static_parallelism=True, k=2))
        t0 = time.time()
        jid = c.networks.train(req)
        st = _wait(c, jid, timeout=200)
        assert st["state"] == "finished", st
        assert time.time() - t0 < 150
        log = c.logs(jid).decode()
        assert "hung collective" in log and "recovering" in log
        assert c.histories.get(jid).data.parallelism == [1.0]
    finally:
        if old is None:
            os.environ.pop("KUBEML_STALL_TIMEOUT", None)
        else:
            os.environ["KUBEML_STALL_TIMEOUT"] = old
        srv.stop()


def test_resume_from_checkpoint(env):
    """A job resumed from another continues its epoch count, history and weights."""
    srv, c, _ = env
    base = TrainRequest(batch_size=64, epochs=1, dataset="mnist", lr=0.05, function_name="lenet",
                        options=TrainOptions(default_parallelism=1, static_parallelism=True, k=-1))
    j1 = c.networks.train(base)
    assert _wait(c, j1)["state"] == "finished"
    h1 = c.histories.get(j1).data
    res = TrainRequest(batch_size=64, epochs=3, dataset="mnist", lr=0.05, function_name="lenet",
                       options=TrainOptions(default_parallelism=1, static_parallelism=True, k=-1, resume_from=j1))
    j2 = c.networks.train(res)
    st = _wait(c, j2)
    assert st["state"] == "finished", st
    h2 = c.histories.get(j2).data
    assert len(h2.train_loss) == 3 and h2.train_loss[0] == h1.train_loss[0]   # carried over + 2 new epochs
    assert h2.train_loss[1] < h1.train_loss[0]                                 # continued, not restarted
    assert h2.epoch_duration == sorted(h2.epoch_duration)
    assert "resuming" in c.logs(j2).decode()


def test_role_clients(env):
    """Internal role clients (reference ml/pkg/ps/client, ml/pkg/train/client) against the
    running server's parameter-server role."""
    from kubeml_amd.control.clients import JobClient, PSClient
    srv, c, _ = env
    assert isinstance(PSClient(srv.url("ps")).list_tasks(), list)
    assert JobClient("http://127.0.0.1:9").health() is False
