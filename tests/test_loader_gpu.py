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


def test_resident_split_holds_only_the_ranks_shard(tmp_path):
    """Each of N workers uploads its own split_minibatches shard, not the whole split (reference
    network.py:263-264); an elastic resize that moves the shard re-uploads just the new one."""
    from kubeml_amd.sdk.loader import ResidentSplit
    from kubeml_amd.sdk.util import split_minibatches
    st, x, y = _store(tmp_path)
    docs = st.num_docs("ds", "train")
    for world in (2, 4):
        for rank in range(world):
            s = ResidentSplit(st, "ds", "train", dev)
            sh = split_minibatches(range(docs), world)[rank]
            s.plan([(d, d + 2) for d in range(sh.start, sh.stop, 2)], 128)
            r0, r1 = sh.start * 64, min(sh.stop * 64, x.shape[0])
            assert (s.w0, s.w1) == (r0, r1) and s.uploaded_rows == r1 - r0 < x.shape[0] // world + 64
            xb, yb = s.next()
            n = min(128, r1 - r0)
            assert np.array_equal(xb.cpu().numpy(), x[r0:r0 + n]) and np.array_equal(yb.cpu().numpy(), y[r0:r0 + n])
    s = ResidentSplit(st, "ds", "train", dev)
    s.plan([(0, 4)], 64)
    s.plan([(1, 3)], 64)                       # inside the window: nothing moves
    assert s.uploaded_rows == 256
    s.plan([(8, 12)], 64)                      # resize moved the shard: new window only
    assert (s.w0, s.w1) == (512, 768) and s.uploaded_rows == 512
    xb, _ = s.next()
    assert np.array_equal(xb.cpu().numpy(), x[512:576])
