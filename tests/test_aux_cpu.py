"""Auxiliary subsystems on CPU: config precedence, tracing, fault injection, checkpoint
layout (torch state_dict names, {jobId}:{name} keys), history / function stores,
metrics exposition names."""
import json
import os

import pytest
import torch


def test_config_env_over_toml(tmp_path, monkeypatch):
    from kubeml_amd.config import Config
    (tmp_path / "kubeml.toml").write_text('controller_port = 12000\nbucket_mb = 32.0\n')
    monkeypatch.setenv("KUBEML_CONFIG", str(tmp_path / "kubeml.toml"))
    monkeypatch.setenv("KUBEML_BUCKET_MB", "16")
    monkeypatch.setenv("DEBUG_ENV", "true")
    c = Config.load()
    assert c.controller_port == 12000 and c.bucket_mb == 16.0 and c.debug_env is True


def test_trace_spans_written(tmp_path):
    from kubeml_amd.utils import trace
    trace.enable(True)
    try:
        trace.set_process("unit", 3)
        with trace.span("epoch", epoch=1):
            with trace.span("iteration", round=0):
                pass
        trace.instant("marker")
        p = trace.flush(str(tmp_path))
    finally:
        trace.enable(False)
    d = json.load(open(p))
    names = [e["name"] for e in d["traceEvents"]]
    assert "epoch" in names and "iteration" in names and "process_name" in names
    assert "rank3" in os.path.basename(p)


def test_fault_rules():
    from kubeml_amd.utils import fault
    fault.configure("raise:at=round:rank=1:round=2")
    fault.point("round", rank=0, round=2)          # other rank: no fault
    fault.point("round", rank=1, round=1)          # other round: no fault
    with pytest.raises(RuntimeError):
        fault.point("round", rank=1, round=2)
    fault.point("round", rank=1, round=2)          # fires once
    fault.configure("")


def test_checkpoint_roundtrip_and_reference_keys(tmp_path):
    from kubeml_amd.models.resnet import resnet20
    from kubeml_amd.nn import flatten_module
    from kubeml_amd.store.ckpt import load_checkpoint, metadata, reference_keys, save_checkpoint, state_dict_cpu
    torch.manual_seed(0)
    m = resnet20()
    flatten_module(m)
    p = save_checkpoint(m, str(tmp_path / "j1.safetensors"), job_id="j1", epoch=3)
    meta = metadata(p)
    assert meta["jobId"] == "j1" and meta["epoch"] == "3"
    m2 = resnet20()
    flatten_module(m2)
    side = load_checkpoint(m2, p)
    assert side["epoch"] == 3
    a, b = state_dict_cpu(m), state_dict_cpu(m2)
    assert a.keys() == b.keys() and all(torch.equal(a[k], b[k]) for k in a)
    keys = reference_keys("j1", a)
    assert "j1:conv1.weight" in keys
    assert "j1:conv1.weight/2" in reference_keys("j1", a, func_id=2)


def test_async_checkpoint_failure_keeps_last_good_file(tmp_path, monkeypatch):
    """A failed background write is reported by the next save() (which still takes and
    writes its own snapshot), and the file on disk stays the last confirmed epoch."""
    import safetensors.torch as st
    from kubeml_amd.store.ckpt import AsyncCheckpointer, load_state, metadata
    m = torch.nn.Linear(4, 3)
    path = str(tmp_path / "j.safetensors")
    ck = AsyncCheckpointer()
    assert ck.save(m, path, job_id="j", epoch=0) is None
    ck.wait()
    assert ck.durable_epoch == 0 and metadata(path)["epoch"] == "0"
    real = st.save_file

    def boom(*a, **k):
        raise OSError("disk full")
    monkeypatch.setattr(st, "save_file", boom)
    with torch.no_grad():
        m.weight.add_(1.0)
    assert ck.save(m, path, job_id="j", epoch=1) is None
    assert isinstance(ck.wait(raise_error=False), OSError)
    assert ck.durable_epoch == 0 and metadata(path)["epoch"] == "0"   # old file intact
    monkeypatch.setattr(st, "save_file", boom)
    ck.save(m, path, job_id="j", epoch=2)                              # fails in background
    monkeypatch.setattr(st, "save_file", real)
    prev = ck.save(m, path, job_id="j", epoch=3)                       # reports it, still writes
    assert isinstance(prev, OSError)
    ck.wait()
    assert ck.durable_epoch == 3 and metadata(path)["epoch"] == "3"
    assert torch.equal(load_state(path)["weight"], m.weight.detach())


def test_history_and_function_stores(tmp_path):
    from kubeml_amd.api.errors import KubeMLException
    from kubeml_amd.api.types import History, JobHistory, TrainRequest
    from kubeml_amd.store.functions import FunctionStore
    from kubeml_amd.store.history import HistoryStore
    hs = HistoryStore(str(tmp_path))
    hs.save(History(id="abc", task=TrainRequest(dataset="d"), data=JobHistory(train_loss=[1.0, 0.5])))
    assert hs.get("abc").data.train_loss == [1.0, 0.5]
    assert [h.id for h in hs.list()] == ["abc"]
    assert hs.prune() == 1 and hs.list() == []
    fs = FunctionStore(str(tmp_path))
    fs.create("f", b"def main():\n    return 1\n")
    assert fs.get("f").environment == "torch" and fs.get("f").concurrency == 50
    with pytest.raises(KubeMLException):
        fs.create("f", b"x = 1\n")
    with pytest.raises(KubeMLException):
        fs.create("bad", b"def (:\n")
    fs.delete("f")
    assert fs.list() == []


def test_metric_names_match_reference():
    from kubeml_amd.api.types import MetricUpdate
    from kubeml_amd.metrics import Metrics
    m = Metrics()
    m.task_started("train")
    m.update("job1", MetricUpdate(validations_loss=0.5, accuracy=90, train_loss=0.7, parallelism=2,
                                  epoch_duration=12))
    text = m.exposition().decode()
    for name in ("kubeml_job_validation_loss", "kubeml_job_validation_accuracy", "kubeml_job_train_loss",
                 "kubeml_job_parallelism", "kubeml_job_epoch_duration_seconds", "kubeml_job_running_total"):
        assert name in text
    assert 'jobid="job1"' in text
    m.clear("job1")
    assert 'jobid="job1"' not in m.exposition().decode()
