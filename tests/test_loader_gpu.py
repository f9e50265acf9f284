"""Pinned streaming loader on the MI355X (sdk/loader.py + csrc/runtime/loader.cpp):
every planned minibatch arrives in HBM byte-exact against ``ShardStore.load_docs``,
in order, across rounds with ragged tails, while the compute stream keeps consuming
earlier batches (device ring reuse is ordered by events)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)


def _store(tmp_path, n=64 * 15 + 37):
    from kubeml_amd.store.shards import ShardStore
    rng = np.random.default_rng(3)
    st = ShardStore(str(tmp_path))
    x = rng.integers(0, 256, (n, 32, 32, 3), dtype=np.uint8)
    y = rng.integers(0, 10, n).astype(np.int64)
    st.create("ds", x, y, x[:300], y[:300])
    return st, x, y


def test_stream_matches_load_docs(tmp_path):
    from kubeml_amd.sdk.loader import SplitStreamer
    st, x, y = _store(tmp_path)
    s = SplitStreamer(st, "ds", "train", dev)
    rounds = [(0, 4), (4, 9), (9, 16)]           # last round has a ragged doc
    bs = 100
    s.plan(rounds, bs)
    acc = torch.zeros((), dtype=torch.float64, device=dev)
    seen = []
    for d0, d1 in rounds:
        ref_x, ref_y = st.load_docs("ds", "train", d0, d1)
        for b0 in range(0, len(ref_x), bs):
            xb, yb = s.next()
            # consume on the compute stream (keeps the ring busy while later copies run)
            acc += xb.double().sum()
            seen.append((xb.clone(), yb.clone(), ref_x[b0:b0 + bs], ref_y[b0:b0 + bs]))
    torch.cuda.synchronize()
    assert s.stream.pending() == 0
    total = 0
    for xb, yb, rx, ry in seen:
        assert xb.shape == rx.shape
        assert np.array_equal(xb.cpu().numpy(), rx)
        assert np.array_equal(yb.cpu().numpy(), ry)
        total += float(rx.astype(np.float64).sum())
    assert float(acc) == total
    # re-plan (new task) with a different batch size while nothing is pending
    s.plan([(2, 3)], 64)
    xb, yb = s.next()
    assert np.array_equal(xb.cpu().numpy(), x[128:192])


@pytest.mark.parametrize("budget_mb", ["8192", "0"])
def test_dataset_resident_or_streamed_matches_load_docs(tmp_path, monkeypatch, budget_mb):
    """KubeDataset's GPU path: a split within KUBEML_RESIDENT_MB is uploaded once and served
    as views (ResidentSplit); a larger one streams through pinned memory (SplitStreamer).
    Both hand out byte-exact batches in plan order."""
    from kubeml_amd.sdk.loader import ResidentSplit, SplitStreamer
    st, x, y = _store(tmp_path)
    monkeypatch.setenv("KUBEML_RESIDENT_MB", budget_mb)

    class DS:
        from kubeml_amd.sdk.dataset import KubeDataset as _K
        _plan_stream = _K._plan_stream
        _stream_ok = lambda self, d: True

    ds = DS()
    ds._store, ds.dataset, ds._streamers = st, "ds", {}
    assert ds._plan_stream("train", [(0, 3), (3, 16)], 128, dev)
    s = ds._streamers["train"]
    assert isinstance(s, ResidentSplit if budget_mb != "0" else SplitStreamer)
    ref_x, ref_y = st.load_docs("ds", "train", 0, 3)
    xb, yb = s.next()
    assert np.array_equal(xb.cpu().numpy(), ref_x[:128]) and np.array_equal(yb.cpu().numpy(), ref_y[:128])
    xb, yb = s.next()
    assert np.array_equal(xb.cpu().numpy(), ref_x[128:192])     # round boundary: ragged batch
